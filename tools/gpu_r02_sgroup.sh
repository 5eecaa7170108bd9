#!/bin/bash
# GPU box: sampler items drawn four per barrier pair — sampler / engine
# tests, then the multi-sample lines and the S = 1 line without prefetch.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_config5_gpu.py -m gpu \
  -x -q --timeout 200 --timeout-method thread > gpurun_out/sg_tests.log 2>&1 || exit $?
rm -f gpurun_out/sg_bench.jsonl
for spec in "cora 8" "cora 16" "citeseer 16"; do
  set -- $spec
  timeout -k 10 300 python bench.py --dataset $1 --samples $2 --steps 100 --warmup 10 --no-cpu-baseline \
    >> gpurun_out/sg_bench.jsonl 2>> gpurun_out/sg_bench.err || exit $?
done
timeout -k 10 200 python bench.py --no-cpu-baseline --no-prefetch-draw >> gpurun_out/sg_bench.jsonl 2>> gpurun_out/sg_bench.err || exit $?
