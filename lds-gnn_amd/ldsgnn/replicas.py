"""Monte-Carlo sample parallelism across GPUs.

Graph samples are independent: every rank runs its own inner chain (own GCN
weights, Adam state and keyed RNG stream: replica = rank) and produces its own
θ-gradient per hyper step.  The only exchange is one all-reduce (mean) of
θ.grad over RCCL/xGMI per hyper step; every rank then applies the identical
SGD + clamp, so θ stays replicated without a broadcast.  One rank = the
reference exactly.

Under the nccl (= RCCL) backend the all-reduce is graph-capturable: the fused
engine then captures it INTO the replayed window graph
(LdsEngine.capture_window reads the reducer's `capturable` attribute), so a
rank replays whole groups of windows as at N = 1 instead of two graphs per
window around an eager collective.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def _group_up() -> bool:
    return dist.is_available() and dist.is_initialized()


def exchange_capturable() -> bool:
    """The exchange can be captured into a HIP graph: no process group (no
    collective at all), or the nccl backend (an RCCL kernel on the capture
    stream).  gloo copies through the host: never captured."""
    if not _group_up():
        return True
    return dist.get_backend() == "nccl"


def allreduce_mean(model: torch.nn.Module) -> None:
    """grad_reducer for OuterProblemTrainer: θ.grad <- mean over ranks (SUM,
    then ÷ world: for the power-of-two world sizes of a node this equals
    scaling each rank's gradient by 1/world exactly)."""
    if not _group_up() or dist.get_world_size() == 1:
        return
    world = dist.get_world_size()
    for p in model.parameters():
        if p.grad is not None:
            dist.all_reduce(p.grad, op=dist.ReduceOp.SUM)
            p.grad.div_(world)


allreduce_mean.capturable = exchange_capturable


def mean_prescale():
    """World size when the mean over ranks may be taken as a SUM of
    gradients each rank has already scaled by 1/world: a process group of
    more than one rank whose size is a power of two (scaling by 2^-k commutes
    with fp32 rounding, so Σ_r (g_r / world) is bit for bit (Σ_r g_r) / world,
    barring subnormals: entries near FLT_MIN may differ by up to
    world · 2^-149, world subnormal ulps).  None otherwise (sum, then divide)."""
    if not _group_up():
        return None
    world = dist.get_world_size()
    return world if world > 1 and world & (world - 1) == 0 else None


def allreduce_sum_(grad: torch.Tensor) -> None:
    """The exchange of a prescaled gradient (mean_prescale): one all-reduce
    SUM, no division pass over θ.grad."""
    if _group_up() and dist.get_world_size() > 1:
        dist.all_reduce(grad, op=dist.ReduceOp.SUM)


def allreduce_mean_always(model: torch.nn.Module) -> None:
    """allreduce_mean that runs the collective at world size 1 too (the
    world-size-1 RCCL rehearsal on one GPU: the same launches as N > 1)."""
    world = dist.get_world_size()
    for p in model.parameters():
        if p.grad is not None:
            dist.all_reduce(p.grad, op=dist.ReduceOp.SUM)
            p.grad.div_(world)


allreduce_mean_always.capturable = exchange_capturable


def collective_capture_probe(device: torch.device) -> bool:
    """Whether every rank can capture an all-reduce into a HIP graph and
    replay it correctly.  Each rank captures a small all-reduce; the ranks
    agree on the outcome with an eager all-reduce BEFORE any replay (a rank
    that failed must not leave the others waiting inside a replayed
    collective), then replay once, check the sum and agree again.  False
    without the nccl backend."""
    if not _group_up() or not exchange_capturable():
        return False
    world = dist.get_world_size()
    ok = True
    x = torch.ones(64, dtype=torch.float32, device=device)
    graph = None
    try:
        graph = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(device)
        s.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(s):
            with torch.cuda.graph(graph, stream=s, capture_error_mode="thread_local"):
                dist.all_reduce(x, op=dist.ReduceOp.SUM)
        torch.cuda.current_stream(device).wait_stream(s)
    except Exception:  # noqa: BLE001  (any capture failure means: do not capture)
        ok = False

    def agree(flag: bool) -> bool:
        t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(int(t.item()))

    if not agree(ok):
        return False
    graph.replay()
    torch.cuda.synchronize(device)
    return agree(bool(torch.all(x == float(world)).item()))
