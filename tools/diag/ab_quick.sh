#!/bin/bash
# GPU box: kernel + engine parity tests, then the bench (real Cora) twice and
# rocprof kernel stats of a short run.  Usage: tools/diag/ab_quick.sh TAG [tests...]
set -o pipefail
tag=$1; shift
sel=${@:-tests/test_kernels_gpu.py tests/test_engine_gpu.py}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest $sel -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1 || exit $?
for i in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --no-breakdown --steps 200 2>/dev/null | tail -1 \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['value']), round(d['steady_state']['value']))" || exit 1
done
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- \
  python3 bench.py --no-cpu-baseline --no-breakdown --steps 100 > gpurun_out/prof_$tag.log 2>&1 || exit 1
