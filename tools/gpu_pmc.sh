#!/bin/bash
# HBM traffic of the engine's kernels from rocprofv3 PMC counters, one counter
# per pass (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950).
# Output: gpurun_out/pmc_<tag>_{fetch,write}/ (CSV).  Summarise with
# tools/pmc_summary.py.
set -o pipefail
tag=${1:-dev}
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  lc=$(echo $c | cut -d_ -f1 | tr 'A-Z' 'a-z')
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc_${tag}_$lc -o run -- \
    python3 bench.py --no-cpu-baseline --steps 50 --warmup 10 > gpurun_out/pmc_${tag}_$lc.log 2>&1 || exit $?
done
