#!/bin/bash
# GPU box: fused θ-grad + draw epilogue drawing four graphs per barrier pair.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu \
  -x -q --timeout 200 --timeout-method thread -k "draw or prefetch or replay" > gpurun_out/fg_tests.log 2>&1 || exit $?
timeout -k 10 120 python tools/microbench/fused_draw.py > gpurun_out/fg_fd.json 2> gpurun_out/fg_fd.err || exit $?
rm -f gpurun_out/fg_bench.jsonl
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline >> gpurun_out/fg_bench.jsonl 2>> gpurun_out/fg_bench.err || exit $?
done
