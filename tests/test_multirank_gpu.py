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


def _worker(rank, world, port, out, per_rank=1):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "lds-gnn_amd")]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ldsgnn.replicas import allreduce_mean
    eng = _trainers(per_rank, rank * per_rank, allreduce_mean)
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


@pytest.mark.parametrize("per_rank", [1, 8])
def test_two_ranks_over_gloo_match_batched_replicas(per_rank):
    """per_rank = 8: BASELINE config 4's split (8 Monte-Carlo samples per
    GPU, replicas 8·rank … 8·rank + 7) against one process batching all 16."""
    world = 2
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    mp.start_processes(_worker, args=(world, _free_port(), out, per_rank), nprocs=world, join=True,
                       start_method="spawn")
    r0, r1 = out[0], out[1]
    eng = _trainers(world * per_rank, 0, None)     # one process, replicas 0 .. world·per_rank - 1 batched
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
        rows.append({"window": w, "ranks_bit_identical": True, f"max_abs_vs_batched_S{world * per_rank}": err})
        assert err < 1e-5, (w, err)
    assert moved > 1e-4
    d = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(d):
        with open(os.path.join(d, f"multirank_gloo_s{per_rank}.json"), "w") as f:
            json.dump({"test": "tests/test_multirank_gpu.py", "world": world, "backend": "gloo (one device)",
                       "samples_per_rank": per_rank,
                       "workload": "cora kNN theta0, tau=5, replica = rank", "theta_moved": moved,
                       "windows": rows}, f, indent=1)


LR_N, LR_SEED, LR_WINDOWS = 1100, 6, 2
# dθ of a dense graph is small (≈ 1/degree): a large outer rate makes θ move
# well past the comparison tolerance in two windows
LR_OUTER = 50.0


def _long_row_problem():
    from tests.parity_harness import synthetic_problem
    from oracle import lds_oracle as O
    prob = synthetic_problem(LR_N, 32, 5, LR_SEED)
    # dense θ ~ U(0, 1): ≈ 550 expected neighbours per row, so the engine takes
    # the long-row (bitmask-aggregation) path by itself, as at config 5
    theta0 = torch.rand(LR_N * (LR_N + 1) // 2, generator=torch.Generator().manual_seed(LR_SEED + 1))
    torch.manual_seed(LR_SEED)
    from ldsgnn.models.gcn import MetaDenseGCN
    gcn = MetaDenseGCN(32, 16, 5, dropout=0.5)
    params = {k: v.detach().clone() for k, v in gcn.named_parameters()}
    return prob, theta0, params, O


def _long_row_worker(rank, world, port, out, kernel, sharded=False):
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "lds-gnn_amd")]
    from collections import OrderedDict

    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import ldsgnn
    from ldsgnn.engine import LdsEngine
    from ldsgnn.replicas import exchange_capturable
    prob, theta0, params, _ = _long_row_problem()
    dev = "cuda"

    def reducer(grad):  # the replicas' all-reduce mean of dθ (800 MB per window at config 5)
        dist.all_reduce(grad, op=dist.ReduceOp.SUM)
        grad.div_(world)
    reducer.capturable = exchange_capturable  # (gloo: not capturable -> split graphs, capture outcome agreed)
    eng = LdsEngine(prob["x"].to(dev), prob["y"].to(dev), prob["train"].to(dev), prob["opt"].to(dev),
                    theta0.clone().to(dev), 5, dropout=0.5, gcn_lr=0.01, gcn_wd=5e-4, outer_lr=LR_OUTER, lr_decay=0.99,
                    tau=5, generator=ldsgnn.rng.Generator(LR_SEED, rank),
                    params=OrderedDict((k, v.to(dev)) for k, v in params.items()), long_rows_kernel=kernel)
    assert eng.long_rows and eng.bitmask_agg == (kernel == "bitmask")
    if sharded:  # band-sharded replicas: factor all-gather, band update, band draws + all-to-all
        from ldsgnn.replicas import BandShards
        sh = BandShards(LR_N)
        eng.set_band_shards(sh)

        def snap():
            eng.sync_theta()
            sh.gather_rows(eng.grad, LR_N)  # (each rank's dθ band)
            return eng.theta.cpu().clone(), eng.grad.cpu().clone()
    else:
        eng.grad_reducer = reducer

        def snap():
            return eng.theta.cpu().clone(), eng.grad.cpu().clone()
    eng.inner_step()
    eng.hyper_step()  # step 0: dθ -> all-reduce -> SGD + clamp (sharded: factors -> band update)
    t0, g0 = snap()
    thetas, grads = [t0], [g0]
    if not sharded:
        head_tail = eng.capture_window(5)
        assert isinstance(head_tail, tuple) and len(head_tail) == 2
    for _ in range(LR_WINDOWS):
        if sharded:
            eng.run_window(5)  # (eager: the sharded exchange is not captured)
        else:
            eng.replay(1)
        torch.cuda.synchronize()
        t, g = snap()
        thetas.append(t)
        grads.append(g)
    eng.check_device_error()
    out[rank] = (thetas, grads)
    dist.destroy_process_group()


@pytest.mark.parametrize("kernel,sharded", [("bitmask", False), ("csr", False), ("bitmask", True), ("csr", True)])
def test_two_ranks_long_row_engine_with_exchange(kernel, sharded):
    """BASELINE config 5's multi-GPU half at a test size: the long-row engine
    (dense θ, n = 1 100, the bitmask aggregation chosen by the engine itself,
    or the CSR spill-pass SpMM) with the replicas' exchange — dθ all-reduced
    (mean) between the split window graphs, or (`sharded`) the band-sharded
    exchange (every rank's factors all-gathered, each rank updating and
    drawing its own row band of θ for every replica, the bands exchanged
    all-to-all; θ gathered for the check) — on two ranks over gloo.  θ is
    bit-identical on both ranks after every window and within 1e-5 of the
    oracle's two replicas updated by their mean hypergradient
    (oracle.replica_hyper_step).  Reference: src/trainers/outer.py:77-84."""
    world = 2
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    mp.start_processes(_long_row_worker, args=(world, _free_port(), out, kernel, sharded), nprocs=world, join=True,
                       start_method="spawn")
    (r0, g0), (r1, g1) = out[0], out[1]
    prob, theta0, params, O = _long_row_problem()
    from collections import OrderedDict
    oracles = [O.LdsProblem(prob["x"], prob["y"], prob["train"], prob["val"], prob["test"], prob["opt"],
                            theta0.clone(), hidden=16, dropout_p=0.5, gcn_lr=0.01, gcn_wd=5e-4, outer_lr=LR_OUTER,
                            lr_decay=0.99, rnd=O.Randomness(LR_SEED, b), params=OrderedDict(params))
               for b in range(world)]
    ref, refg = [], []
    for w in range(LR_WINDOWS + 1):
        for _ in range(1 if w == 0 else 5):
            for orc in oracles:
                orc.inner_step(orc.sample())
        refg.append(O.replica_hyper_step(oracles)[1])
        ref.append(oracles[0].theta.detach().clone())
    rows = []
    for w, (a, b, c, ga, gb, gc) in enumerate(zip(r0, r1, ref, g0, g1, refg)):
        assert torch.equal(a, b) and torch.equal(ga, gb), w
        err = float((a - c).abs().max())
        grel = float((ga - gc).abs().max() / gc.abs().max())
        rows.append({"window": w, "ranks_bit_identical": True, "max_abs_theta_vs_oracle_replica_mean": err,
                     "max_grad_rel_vs_oracle_replica_mean": grel})
        assert err < 1e-5, (w, err)
        assert grel < 1e-4, (w, grel)  # (the windows' Adam steps: test_engine_long_rows_match_oracle's bound)
    assert float((ref[-1] - theta0).abs().max()) > 1e-3
    d = os.path.join(ROOT, "gpurun_out")
    if os.path.isdir(d):
        tag = "sharded" if sharded else "allreduce"
        with open(os.path.join(d, f"multirank_gloo_long_rows_{kernel}_{tag}.json"), "w") as f:
            json.dump({"test": "tests/test_multirank_gpu.py::test_two_ranks_long_row_engine_with_exchange",
                       "world": world, "backend": "gloo (one device)", "n": LR_N, "kernel": kernel,
                       "exchange": "band-sharded (factor all-gather, band update, band draws + all-to-all)"
                       if sharded else "dense dθ all-reduce (mean)",
                       "windows": rows}, f, indent=1)
