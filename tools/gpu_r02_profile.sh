#!/bin/bash
# GPU box: the default bench line, its rocprofv3 kernel-trace summary and the
# two PMC traffic passes (FETCH_SIZE, WRITE_SIZE: one TCC counter set each).
# Usage: tools/gpu_r02_profile.sh TAG
set -o pipefail
tag=${1:-r02}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- \
  python3 bench.py --no-cpu-baseline --steps 100 > gpurun_out/prof_$tag.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  lc=$(echo $c | cut -d_ -f1 | tr 'A-Z' 'a-z')
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc_${tag}_$lc -o run -- \
    python3 bench.py --no-cpu-baseline --no-breakdown --steps 50 --warmup 10 > gpurun_out/pmc_${tag}_$lc.log 2>&1 || exit $?
done
