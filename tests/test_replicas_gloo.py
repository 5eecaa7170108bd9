"""N>1 path on CPU: two gloo ranks average θ.grad exactly as the RCCL path
does (ldsgnn.replicas.allreduce_mean, the engine reducer in bench.py), so θ
stays identical on every rank after the SGD step.  world_size 2, 127.0.0.1."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ldsgnn.replicas import allreduce_mean
    torch.manual_seed(0)
    theta = torch.nn.Parameter(torch.rand(55))           # same θ on every rank
    g = torch.Generator().manual_seed(100 + rank)        # each replica: own sample -> own gradient
    theta.grad = torch.randn(55, generator=g)
    model = torch.nn.Module()
    model.theta = theta
    allreduce_mean(model)
    with torch.no_grad():                                 # SGD + clamp, identical on every rank
        theta.add_(theta.grad, alpha=-0.1).clamp_(0, 1)
    out[rank] = theta.detach().clone()
    dist.destroy_process_group()


def test_two_replicas_average_and_stay_in_sync():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    g0 = torch.randn(55, generator=torch.Generator().manual_seed(100))
    g1 = torch.randn(55, generator=torch.Generator().manual_seed(101))
    torch.manual_seed(0)
    theta = torch.rand(55)
    want = (theta - 0.1 * (g0 + g1) / 2).clamp(0, 1)
    assert torch.allclose(out[0], out[1], atol=0) and torch.allclose(out[0], want, atol=1e-7)


def _prescale_worker(rank, world, port, out, subnormal=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ldsgnn.replicas import allreduce_mean, allreduce_sum_, mean_prescale
    g = torch.Generator().manual_seed(200 + rank)
    grad = torch.randn(4099, generator=g) * torch.logspace(-20, 20, 4099)
    if subnormal:  # around FLT_MIN: normal and subnormal dθ entries
        grad = torch.randn(4099, generator=g) * (2.0 ** -126) * torch.logspace(-6, 1, 4099)
    model = torch.nn.Module()
    model.theta = torch.nn.Parameter(torch.zeros(4099))
    model.theta.grad = grad.clone()
    allreduce_mean(model)                     # SUM, then ÷ world
    w = mean_prescale()
    pre = grad * (1.0 / w)                    # what the engine's assembly writes (gscale = 1/world)
    allreduce_sum_(pre)                       # SUM alone
    out[rank] = (w, model.theta.grad.clone(), pre)
    dist.destroy_process_group()


def test_prescaled_sum_equals_mean_bit_for_bit():
    """The engine's prescaled exchange (dθ assembled × 1/world, then one
    all-reduce SUM: LdsEngine._prescale, ldsgnn.fused) gives the bits of
    allreduce_mean's SUM-then-divide for a power-of-two world."""
    from ldsgnn.replicas import mean_prescale
    assert mean_prescale() is None  # no process group: no prescaling
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_prescale_worker, args=(world, port, out), nprocs=world, join=True)
    for r in range(world):
        w, mean, pre = out[r]
        assert w == world
        assert torch.equal(mean, pre)


def test_prescaled_sum_near_flt_min_within_one_subnormal_ulp():
    """Round-5 ADVICE: scaling by 2^-k is exact only above the subnormal
    range, so for dθ entries near FLT_MIN the prescaled exchange may differ
    from SUM-then-divide.  Bounded: each rank's g/world rounds once (half a
    subnormal ulp each) and the divide once, so |difference| <= world · 2^-149
    (2^-149: one ulp of the subnormal range, far below any θ step lr·dθ can
    make visible), as documented at ldsgnn.fused.engine_from_trainers."""
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_prescale_worker, args=(world, port, out, True), nprocs=world, join=True)
    for r in range(world):
        w, mean, pre = out[r]
        diff = (mean.double() - pre.double()).abs()
        assert float(diff.max()) <= world * 2.0 ** -149, float(diff.max())
        assert float(diff.max()) > 0.0  # (the case the bound is about does occur)
