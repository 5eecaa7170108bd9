#!/bin/bash
# Config 5 after the bitmask-aggregation split-sum fold: the aggregation and
# config-5 tests, the config-5 bench line (window breakdown with the bitmask
# aggregation's int8-MFMA roofline), its kernel-trace summary.
# Usage: tools/gpu_r02_config5.sh TAG
set -o pipefail
tag=${1:-r02}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_config5_gpu.py -k "bitmask or config5 or n20000" \
  -x -v --timeout 200 --timeout-method thread > gpurun_out/c5_tests_$tag.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --dataset synthetic20k --steps 10 --warmup 5 --no-cpu-baseline \
  > gpurun_out/c5_bench_$tag.json 2> gpurun_out/c5_bench_$tag.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5_prof_$tag -o run -- \
  python3 bench.py --dataset synthetic20k --steps 10 --warmup 5 --no-cpu-baseline --no-breakdown \
  > gpurun_out/c5_prof_$tag.log 2>&1 || exit $?
