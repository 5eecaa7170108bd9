#!/bin/bash
# GPU box: one SQ counter pass over a short default bench (issue / wait breakdown per kernel).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
  --kernel-trace --output-format csv -d gpurun_out/pmc_sq -o run -- \
  python3 bench.py --no-cpu-baseline --no-breakdown --steps 20 --warmup 10 > gpurun_out/pmc_sq.log 2>&1 || exit $?
