#!/bin/bash
# GPU box: θ-grad tile form at the multi-sample shapes (Cora S = 8, 16;
# Citeseer S = 16): the shape-picked default (128-tiles for k >= 1024) against
# the 64-tile 16-wide-chunk grouped form.
set -o pipefail
mkdir -p gpurun_out
for form in bf16x3 bf16x3-t64k16-grouped; do
  for spec in "cora 8" "cora 16" "citeseer 16"; do
    set -- $spec
    timeout -k 10 300 python bench.py --dataset $1 --samples $2 --steps 50 --warmup 10 --no-cpu-baseline \
      --theta-form $form > gpurun_out/tf_${form}_${1}_$2.json 2> gpurun_out/tf_${form}_${1}_$2.err || exit $?
  done
done
