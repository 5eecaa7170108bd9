#!/bin/bash
# GPU box, end of round 2: the whole -m gpu suite, smoke(), the default bench
# line, its rocprofv3 kernel-trace summary, the two PMC traffic passes, the
# config-5 bench line.  Usage: tools/gpu_r02_final.sh TAG
set -o pipefail
tag=${1:-r02final}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_$tag.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$tag.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- \
  python3 bench.py --no-cpu-baseline --steps 100 > gpurun_out/prof_$tag.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  lc=$(echo $c | cut -d_ -f1 | tr 'A-Z' 'a-z')
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc_${tag}_$lc -o run -- \
    python3 bench.py --no-cpu-baseline --no-breakdown --steps 50 --warmup 10 > gpurun_out/pmc_${tag}_$lc.log 2>&1 || exit $?
done
timeout -k 10 400 python -u bench.py --dataset synthetic20k --steps 10 --warmup 5 --no-cpu-baseline \
  > gpurun_out/c5_bench_$tag.json 2> gpurun_out/c5_bench_$tag.err || exit $?
