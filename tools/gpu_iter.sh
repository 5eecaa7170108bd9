#!/bin/bash
# Development iteration on the GPU box: engine tests, S=1 and S=16 bench lines, S=16 kernel profile.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_iter.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/b_s1.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline --samples 16 > gpurun_out/b_s16.log 2>&1 || exit $?
bash tools/gpu_prof.sh s16 --samples 16 || exit $?
