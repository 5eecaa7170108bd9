#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_bench_gpu.py -m gpu -x -v --timeout 600 --timeout-method thread \
  > gpurun_out/bt_tests.log 2>&1 || exit $?
