#!/bin/bash
# GPU box: the θ-grad + next-window draw fusion — equivalence test, chain
# timing, kernel-trace summary.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "sgd_draw or theta_grad" > gpurun_out/fd_tests.log 2>&1 || exit $?
timeout -k 10 120 python tools/microbench/fused_draw.py > gpurun_out/fd.json 2> gpurun_out/fd.err || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fd_prof -o run -- \
  python3 tools/microbench/fused_draw.py > gpurun_out/fd_prof.log 2>&1 || exit $?
