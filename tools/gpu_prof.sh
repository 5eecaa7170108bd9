#!/bin/bash
# rocprofv3 kernel-trace summary of a bench configuration: tools/gpu_prof.sh TAG [bench args...]
set -o pipefail
tag=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- \
  python3 bench.py --no-cpu-baseline --steps 100 "$@" > gpurun_out/p_$tag.log 2>&1 || exit $?
