#!/bin/bash
# GPU box: the whole -m gpu suite with the pipelined θ-grad in the by-shape
# rule, then the multi-sample bench lines (Cora S = 8 / 16, Citeseer S = 16).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pipe_e2e_tests.log 2>&1 || exit $?
for spec in "cora 8" "cora 16" "citeseer 16"; do
  set -- $spec
  timeout -k 10 300 python bench.py --dataset $1 --samples $2 --steps 100 --warmup 10 --no-cpu-baseline \
    > gpurun_out/pe_${1}_$2.json 2> gpurun_out/pe_${1}_$2.err || exit $?
done
