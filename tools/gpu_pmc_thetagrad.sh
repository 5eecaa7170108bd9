#!/bin/bash
# SQ counters of the split-bf16 θ-grad kernels at Cora S = 1 and config 5
# (tools/thetagrad_forms.py restricted to the default forms).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
export THETA_FORMS=bf16x3-t64k16-grouped,bf16x3-t128-grouped
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --kernel-trace --output-format csv -d gpurun_out/pmc_tg_sq -o run -- python3 tools/thetagrad_forms.py cora-S1 synthetic20k-S1 > gpurun_out/pmc_tg_sq.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d gpurun_out/pmc_tg_sq2 -o run -- python3 tools/thetagrad_forms.py cora-S1 synthetic20k-S1 > gpurun_out/pmc_tg_sq2.log 2>&1 || exit $?
