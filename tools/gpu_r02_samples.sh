#!/bin/bash
# GPU box: the multi-sample configs (BASELINE 3 / 4 shapes) on the round-2
# engine: Cora S = 8 and 16, Citeseer S = 16, each with its window breakdown,
# and a kernel-trace summary of the Citeseer S = 16 run.  Usage: TAG
set -o pipefail
tag=${1:-r02}
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "cora 8" "cora 16" "citeseer 16"; do
  set -- $spec
  timeout -k 10 300 python bench.py --dataset $1 --samples $2 --steps 100 --warmup 10 --no-cpu-baseline \
    > gpurun_out/s_${1}_$2_$tag.json 2> gpurun_out/s_${1}_$2_$tag.err || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s_prof_$tag -o run -- \
  python3 bench.py --dataset citeseer --samples 16 --steps 50 --warmup 10 --no-cpu-baseline --no-breakdown \
  > gpurun_out/s_prof_$tag.log 2>&1 || exit $?
