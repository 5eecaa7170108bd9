#!/bin/bash
# GPU box: θ-grad form 8 (software-pipelined 128-tile) — parity tests, then
# timing against the 64- and 128-tile forms at the engine's shapes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "theta_grad" > gpurun_out/pipe_tests.log 2>&1 || exit $?
THETA_FORMS=${FORMS:-bf16x3-t64k16-grouped,bf16x3-t128-grouped,bf16x3-t128-pipe} timeout -k 10 300 \
  python tools/thetagrad_forms.py ${SHAPES:-cora-S1 cora-S16 citeseer-S16 synthetic20k-S1} > gpurun_out/pipe_forms.jsonl 2> gpurun_out/pipe_forms.err || exit $?
