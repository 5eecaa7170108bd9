#!/bin/bash
# GPU box: the whole -m gpu suite, smoke(), and the GAE-with-proposal-dropout
# engine bench next to the drop-in path.  Usage: tools/gpu_r02_suite.sh TAG
set -o pipefail
tag=${1:-r02}
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/gpu_tests_$tag.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$tag.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --graph-model gae --gae-dropout 0.5 --steps 50 --warmup 10 --no-cpu-baseline \
  --no-breakdown > gpurun_out/gae_drop_engine_$tag.json 2> gpurun_out/gae_drop_engine_$tag.err || exit $?
timeout -k 10 300 python bench.py --graph-model gae --gae-dropout 0.5 --path autograd --steps 20 --warmup 5 \
  --no-cpu-baseline --no-breakdown > gpurun_out/gae_drop_dropin_$tag.json 2> gpurun_out/gae_drop_dropin_$tag.err || exit $?
