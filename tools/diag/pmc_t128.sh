#!/bin/bash
# GPU box: SQ issue / LDS / MFMA counters of the 128-tile θ-grad assembly at
# Cora S = 8 (the per-rank shape of BASELINE config 4): two passes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES \
  --kernel-trace --output-format csv -d gpurun_out/pmc_t128a -o run -- \
  python3 bench.py --samples 8 --no-cpu-baseline --no-breakdown --steps 20 --warmup 10 > gpurun_out/pmc_t128a.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD \
  --kernel-trace --output-format csv -d gpurun_out/pmc_t128b -o run -- \
  python3 bench.py --samples 8 --no-cpu-baseline --no-breakdown --steps 20 --warmup 10 > gpurun_out/pmc_t128b.log 2>&1 || exit $?
