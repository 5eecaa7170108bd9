"""Monte-Carlo sample parallelism across GPUs.

Graph samples are independent: every rank runs its own inner chain (own GCN
weights, Adam state and keyed RNG stream: replica = rank) and produces its own
θ-gradient per hyper step.  The only exchange is one all-reduce (mean) of
θ.grad over RCCL/xGMI per hyper step; every rank then applies the identical
SGD + clamp, so θ stays replicated without a broadcast.  One rank = the
reference exactly.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def allreduce_mean(model: torch.nn.Module) -> None:
    """grad_reducer for OuterProblemTrainer: θ.grad <- mean over ranks."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    world = dist.get_world_size()
    for p in model.parameters():
        if p.grad is not None:
            dist.all_reduce(p.grad, op=dist.ReduceOp.SUM)
            p.grad.div_(world)
