#!/bin/bash
# GPU-box perf iteration: engine parity tests, bench on the real and synthetic
# Cora workloads, per-launch chain microbench.  Usage: tools/gpu_perf.sh [tests...]
set -o pipefail
mkdir -p gpurun_out
sel=${@:-tests/test_engine_gpu.py tests/test_workloads_gpu.py}
timeout -k 10 900 python -u -m pytest $sel -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1 || exit $?
for ds in cora cora-synthetic; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --dataset $ds --steps 100 > gpurun_out/perf_$ds.json 2>/dev/null || exit $?
done
timeout -k 10 240 python tools/microbench/kernel_chain.py > gpurun_out/kchain.jsonl 2> gpurun_out/kchain.err || exit $?
