#!/bin/bash
# GPU box: prefetched window draws (θ-grad kernel draws the next window's
# graphs) — engine / kernel tests, then the bench with and without it.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/pf_tests.log 2>&1 || exit $?
rm -f gpurun_out/pf_bench.jsonl
for a in "" "--no-prefetch-draw" "" "--no-prefetch-draw"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline $a >> gpurun_out/pf_bench.jsonl 2>> gpurun_out/pf_bench.err || exit $?
done
