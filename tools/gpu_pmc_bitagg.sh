#!/bin/bash
# PMC passes over the config-5 aggregation tool (tools/spmm_config5.py):
# MFMA / VALU / LDS activity of bitagg_main_kernel, then its HBM bytes.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU --kernel-trace --output-format csv -d gpurun_out/pmc_bitagg_sq -o run -- python3 tools/spmm_config5.py > gpurun_out/pmc_bitagg_sq.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_bitagg_fetch -o run -- python3 tools/spmm_config5.py > gpurun_out/pmc_bitagg_fetch.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_bitagg_write -o run -- python3 tools/spmm_config5.py > gpurun_out/pmc_bitagg_write.log 2>&1 || exit $?
