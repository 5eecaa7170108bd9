#!/bin/bash
# GPU box: the fused-runner tests, then accuracy on the real Planetoid splits
# with the fused runner (per-step HIP graphs (the default), tau = 20), final round-2 code.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "runner" > gpurun_out/accg_tests.log 2>&1 || exit $?
rm -f gpurun_out/acc_r02g.jsonl
for ds in cora citeseer; do
  timeout -k 10 400 python -u tools/accuracy_run.py --dataset $ds --seeds 5 --tau 20 --fused \
    >> gpurun_out/acc_r02g.jsonl 2>> gpurun_out/acc_r02g.err || exit $?
done
