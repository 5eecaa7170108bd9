#!/bin/bash
# Rehearse the N>1 bench path on a one-GPU box: 2 ranks share the card over
# the gloo backend (RCCL refuses two ranks on one device).  Same code path as
# the driver's RCCL run except the collective's transport.  Second run: config
# 4's layout (replica samples per rank, here 8 per rank).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --backend gloo --steps 50 --warmup 10 --no-cpu-baseline \
  > gpurun_out/bench_2rank_gloo.log 2>&1 || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29518 bench.py --gpus 2 --backend gloo --samples 8 --steps 50 --warmup 10 --no-cpu-baseline \
  > gpurun_out/bench_2rank_gloo_s8.log 2>&1 || exit $?
