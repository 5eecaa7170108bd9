"""The N > 1 path on the GPU: two ranks (processes) over gloo on one device,
each running the fused engine with its Monte-Carlo replica (replica = rank)
and the trainer's grad_reducer (ldsgnn.replicas.allreduce_mean of θ.grad),
the window captured as two HIP graphs split at the exchange — exactly what
bench.py runs per GPU under torchrun.  Checks:

  * θ is bit-identical on both ranks after every window (every rank applies
    the same averaged update);
  * θ equals a single-process engine batching the same two replicas
    (S = 2, mean hypergradient in one rank-2K assembly) within 1e-5.

SURVEY §8(e); the reference only fans out independent jobs
(/root/reference/configs/seml/final/lds.yaml:1-13).  A summary goes to
gpurun_out/multirank_gloo.json when that directory exists."""
import json
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEED, WINDOWS = 23, 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _trainers(samples, replica0, reducer):
    import numpy as np

    import ldsgnn
    from ldsgnn.data.workloads import load_workload
    from ldsgnn.models.gcn import MetaDenseGCN
    from ldsgnn.models.graph import BernoulliGraphModel
    from ldsgnn.trainers.inner import InnerProblemTrainer
    from ldsgnn.trainers.outer import OuterProblemTrainer
    from ldsgnn.utils.graph import split_mask
    data = load_workload("cora")
    np.random.seed(SEED)
    data.val_mask, opt = split_mask(data.val_mask, 0.5, shuffle=True)
    data = data.to("cuda")
    ldsgnn.rng.manual_seed(SEED, replica0)
    torch.manual_seed(SEED)
    gcn = MetaDenseGCN(data.num_features, 16, data.num_classes, dropout=0.5).to("cuda")
    inner = InnerProblemTrainer(gcn, data, lr=0.01, weight_decay=5e-4)
    gm = BernoulliGraphModel(data.dense_adj)
    outer = OuterProblemTrainer(torch.optim.SGD(gm.parameters(), lr=0.1), data, opt.to("cuda"), gm,
                                lr_decay=0.99, grad_reducer=reducer)
    from ldsgnn.fused import engine_from_trainers
    return engine_from_trainers(inner, outer, tau=5, generator=ldsgnn.rng.default_generator, samples=samples)


def _worker(rank, world, port, out):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "lds-gnn_amd")]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ldsgnn.replicas import allreduce_mean
    eng = _trainers(1, rank, allreduce_mean)
    assert eng.grad_reducer is not None
    eng.inner_step()
    eng.hyper_step()            # step 0: dθ → all-reduce → SGD
    head_tail = eng.capture_window(5)  # split at the exchange (the engine's reducer)
    assert isinstance(head_tail, tuple) and len(head_tail) == 2
    thetas = [eng.theta.cpu().clone()]
    for _ in range(WINDOWS):
        eng.replay(1)
        torch.cuda.synchronize()
        thetas.append(eng.theta.cpu().clone())
    out[rank] = thetas
    dist.destroy_process_group()


def test_two_ranks_over_gloo_match_batched_replicas():
    world = 2
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(world, _free_port(), out), nprocs=world, join=True, start_method="spawn")
    r0, r1 = out[0], out[1]
    eng = _trainers(2, 0, None)     # one process, replicas 0 and 1 batched
    eng.inner_step()
    eng.hyper_step()
    ref = [eng.theta.cpu().clone()]
    eng.capture_window(5)
    for _ in range(WINDOWS):
        eng.replay(1)
        torch.cuda.synchronize()
        ref.append(eng.theta.cpu().clone())
    moved = float((ref[-1] - ref[0]).abs().max())
    rows = []
    for w, (a, b, c) in enumerate(zip(r0, r1, ref)):
        assert torch.equal(a, b), w                      # replicas in sync, bit for bit
        err = float((a - c).abs().max())
        rows.append({"window": w, "ranks_bit_identical": True, "max_abs_vs_batched_S2": err})
        assert err < 1e-5, (w, err)
    assert moved > 1e-4
    d = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(d):
        with open(os.path.join(d, "multirank_gloo.json"), "w") as f:
            json.dump({"test": "tests/test_multirank_gpu.py", "world": world, "backend": "gloo (one device)",
                       "workload": "cora kNN theta0, tau=5, replica = rank", "theta_moved": moved,
                       "windows": rows}, f, indent=1)
