#!/bin/bash
# Round-end validation on one MI355X: every GPU test, smoke(), the PMC traffic
# passes (their summary becomes the record bench.py reads for roofline.traffic),
# the default bench line (with the CPU baseline), its kernel-trace profile, and
# the 2-rank rehearsal.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final_tests.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || exit $?
bash tools/gpu_pmc.sh final || exit $?
python tools/pmc_summary.py gpurun_out/pmc_final --json gpurun_out/pmc_traffic_final.json > gpurun_out/pmc_traffic_final.txt || exit $?
cp gpurun_out/pmc_traffic_final.json profiles/r01_pmc_traffic.json || exit $?
timeout -k 10 400 python bench.py > gpurun_out/final_bench.log 2>&1 || exit $?
bash tools/gpu_prof.sh final || exit $?
bash tools/gpu_multirank.sh || exit $?
