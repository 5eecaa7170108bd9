#!/bin/bash
# Each graph generative model on the Cora-shaped config: LDS Bernoulli θ, the
# embedding model, the GAE model — on the drop-in (autograd) trainers and on
# the fused engine (embedding / GAE: θ = P(parameters), eager windows).
set -o pipefail
mkdir -p gpurun_out
for m in lds embedding gae; do
  timeout -k 10 300 python -u bench.py --path autograd --graph-model $m --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b_gm_$m.log 2>&1 || exit $?
  timeout -k 10 300 python -u bench.py --path engine --graph-model $m --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/b_gm_eng_$m.log 2>&1 || exit $?
done
