#!/bin/bash
# Drop-in (autograd) path with each graph generative model on the Cora-shaped
# config: LDS Bernoulli θ, the embedding model, the GAE model.
set -o pipefail
mkdir -p gpurun_out
for m in lds embedding gae; do
  timeout -k 10 300 python -u bench.py --path autograd --graph-model $m --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b_gm_$m.log 2>&1 || exit $?
done
