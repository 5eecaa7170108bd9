#!/bin/bash
# GPU box: kernel-trace summaries of config 3 (Citeseer S = 16) and config 5
# (n = 20 000) on the final round-2 code.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cp_cite -o run -- \
  python3 bench.py --dataset citeseer --samples 16 --steps 50 --warmup 10 --no-cpu-baseline --no-breakdown \
  > gpurun_out/cp_cite.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cp_c5 -o run -- \
  python3 bench.py --dataset synthetic20k --steps 10 --warmup 5 --no-cpu-baseline --no-breakdown \
  > gpurun_out/cp_c5.log 2>&1 || exit $?
