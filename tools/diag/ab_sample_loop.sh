#!/bin/bash
# GPU box: sampler parity tests, then the bench with the window's graphs drawn
# one block per (tile, graph) (0) or looping over one θ load per tile (1), and
# rocprof kernel stats + FETCH_SIZE of both.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit $?
for v in 0 1 0 1; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-breakdown --steps 200 --sample-loop $v 2>/dev/null | tail -1 \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('loop=$v', round(d['value']), round(d['steady_state']['value']))" || exit 1
done
export TMPDIR=/tmp
for v in 0 1; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_loop$v -o run -- \
    python3 bench.py --no-cpu-baseline --no-breakdown --steps 100 --sample-loop $v > gpurun_out/prof_loop$v.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_loop${v}_fetch -o run -- \
    python3 bench.py --no-cpu-baseline --no-breakdown --steps 50 --warmup 10 --sample-loop $v > gpurun_out/pmc_loop${v}_fetch.log 2>&1 || exit 1
done
