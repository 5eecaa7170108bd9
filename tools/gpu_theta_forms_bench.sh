#!/bin/bash
# θ-grad assembly forms end to end: the whole GPU suite, then bench lines with
# the default (split-bf16, by shape) and the fp32-MFMA form at Cora S = 1,
# Cora S = 16, Citeseer S = 16 and config 5.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tf_tests.log 2>&1 || exit $?
B="timeout -k 10 300 python -u bench.py --no-cpu-baseline"
for form in bf16x3 fp32; do
  $B --theta-form $form > gpurun_out/tf_cora_s1_$form.log 2>&1 || exit $?
  $B --theta-form $form --samples 16 --steps 100 --warmup 10 > gpurun_out/tf_cora_s16_$form.log 2>&1 || exit $?
  $B --theta-form $form --dataset citeseer --samples 16 --steps 50 --warmup 10 > gpurun_out/tf_cite_s16_$form.log 2>&1 || exit $?
  $B --theta-form $form --dataset synthetic20k --steps 10 --warmup 5 > gpurun_out/tf_c5_$form.log 2>&1 || exit $?
done
