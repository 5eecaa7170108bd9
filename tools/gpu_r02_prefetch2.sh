#!/bin/bash
# GPU box: prefetched draws on the exchange path (SGD + clamp fused with the
# next window's draw) — engine / kernel / multirank tests, 2-rank rehearsal.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py tests/test_kernels_gpu.py tests/test_multirank_gpu.py -m gpu \
  -x -q --timeout 200 --timeout-method thread > gpurun_out/pf2_tests.log 2>&1 || exit $?
bash tools/gpu_multirank.sh || exit $?
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29519 bench.py --gpus 2 --backend gloo --steps 50 --warmup 10 --no-cpu-baseline --no-prefetch-draw \
  --strong-total 0 > gpurun_out/bench_2rank_gloo_nopf.log 2>&1 || exit $?
