#!/bin/bash
# GPU box: τ-windows per captured HIP graph (1, 2, 4, 8) at the bench default.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 60 --timeout-method thread \
  -k "replay" > gpurun_out/gwin_tests.log 2>&1 || exit $?
for w in 1 2 4 8 1; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-breakdown --graph-windows $w >> gpurun_out/gwin.jsonl 2>> gpurun_out/gwin.err || exit $?
done
