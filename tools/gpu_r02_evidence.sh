#!/bin/bash
# GPU box: the pretrainer golden test, the phase-boundary microbench (graph
# launch vs grid barrier), the sampler degree-count A/B under rocprofv3, and
# the default bench line (now with the committed PMC record for `traffic`).
# Usage: tools/gpu_r02_evidence.sh TAG
set -o pipefail
tag=${1:-r02c}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_golden_gpu.py -k pretrainer -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/pretrainer_$tag.log 2>&1 || exit $?
timeout -k 10 60 tools/microbench/grid_barrier > gpurun_out/grid_barrier_$tag.jsonl 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sdeg_$tag -o run -- \
  python3 tools/diag/sampler_deg_ab.py > gpurun_out/sdeg_$tag.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || exit $?
