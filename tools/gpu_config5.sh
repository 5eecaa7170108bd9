#!/bin/bash
# Config 5 (synthetic N = 20 000, dense θ ~ U(0,1)) through the fused engine:
# long-row parity tests, then bench lines (default: bitmask aggregation) with
# the θ-grad and aggregation roofline legs, and a kernel-trace profile.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -q -k long_rows --timeout 200 --timeout-method thread > gpurun_out/t_long.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --dataset synthetic20k --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/b_c5.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --dataset synthetic20k --steps 10 --warmup 5 --no-cpu-baseline --kernel lds_aggregate_bitmask > gpurun_out/b_c5_agg.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python3 bench.py --dataset synthetic20k --steps 10 --warmup 5 --no-cpu-baseline > gpurun_out/p_c5.log 2>&1 || exit $?
