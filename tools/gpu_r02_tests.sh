#!/bin/bash
# GPU box: the whole -m gpu suite, smoke(), and the two diagnostics that steer
# the next changes (sampler Philox decisions, graph-branch concurrency).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 60 python tools/microbench/graph_branches.py > gpurun_out/graph_branches.json 2> gpurun_out/graph_branches.err || exit $?
timeout -k 10 120 python tools/diag/theta_quads.py > gpurun_out/theta_quads.jsonl 2> gpurun_out/theta_quads.err || exit $?
