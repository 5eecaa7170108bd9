#!/bin/bash
# GPU-box check: the -m gpu suite, the default bench line, the per-launch chain
# microbench.  Usage: tools/gpu_check.sh [pytest selector...]
set -o pipefail
mkdir -p gpurun_out
sel=${@:-tests}
timeout -k 10 900 python -u -m pytest $sel -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench_full.log 2>&1 || exit $?
timeout -k 10 240 python tools/microbench/kernel_chain.py > gpurun_out/kchain.jsonl 2> gpurun_out/kchain.err || exit $?
