#!/bin/bash
# GPU-box check used during development: engine + kernel parity tests, the
# default bench line and a kernel-trace profile (tag = $1).
set -o pipefail
tag=${1:-dev}
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -x -q > gpurun_out/t_engine.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/b_$tag.log 2>&1 || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python3 bench.py --no-cpu-baseline --steps 100 > gpurun_out/p_$tag.log 2>&1 || exit $?
