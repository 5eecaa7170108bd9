#!/bin/bash
# GPU box: LDS / MFMA SQ counters over a short default bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES \
  --kernel-trace --output-format csv -d gpurun_out/pmc_sq2 -o run -- \
  python3 bench.py --no-cpu-baseline --no-breakdown --steps 20 --warmup 10 > gpurun_out/pmc_sq2.log 2>&1 || exit $?
