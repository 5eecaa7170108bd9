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
