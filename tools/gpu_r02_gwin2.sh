#!/bin/bash
# GPU box: grouped-window replay tests, the default bench line (4 windows per
# graph), the driver's short invocation, and the 2-rank gloo rehearsal.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 60 --timeout-method thread \
  -k "replay" > gpurun_out/gwin2_tests.log 2>&1 || exit $?
timeout -k 10 200 python bench.py > gpurun_out/gwin2_bench.json 2> gpurun_out/gwin2_bench.err || exit $?
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/gwin2_driver.json 2> gpurun_out/gwin2_driver.err || exit $?
bash tools/gpu_multirank.sh || exit $?
