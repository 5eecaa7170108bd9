"""Build the fused engine from the drop-in trainers (same problem, same state).

`engine_from_trainers(inner, outer)` maps an InnerProblemTrainer
(MetaDenseGCN + differentiable Adam) and an OuterProblemTrainer
(BernoulliGraphModel + plain SGD, optional StepLR) onto an LdsEngine that
updates the graph model's θ in place and continues the trainers' RNG stream.
"""
from __future__ import annotations

from . import rng as _rng
from .engine import LdsEngine


def engine_from_trainers(inner, outer, tau: int = 5, generator: "_rng.Generator" = None,
                         samples: int = 1) -> LdsEngine:
    """samples > 1: S replica chains (replicas generator.replica + b) batched
    in one engine; θ moves by their mean hypergradient."""
    from .models.graph import BernoulliGraphModel
    gm = outer.model
    if not isinstance(gm, BernoulliGraphModel) or gm.directed:
        raise NotImplementedError("the fused engine implements the undirected LDS Bernoulli model")
    opt = outer.optimizer
    if len(opt.param_groups) != 1:
        raise NotImplementedError("one θ parameter group expected")
    grp = opt.param_groups[0]
    if grp.get("momentum", 0) or grp.get("weight_decay", 0) or grp.get("nesterov", False) or \
            grp.get("dampening", 0):
        raise NotImplementedError("the fused engine implements plain SGD on θ")
    if outer.lr_decay is not None and outer.lr_decay_step_size != 1:
        raise NotImplementedError("StepLR with step_size 1 only")
    gcn = inner.model
    data = inner.data
    return LdsEngine(data.x, data.y, data.train_mask, outer.opt_mask, gm.probs.data, data.num_classes,
                     dropout=gcn.dropout, gcn_lr=inner.lr, gcn_wd=inner.weight_decay, outer_lr=grp["lr"],
                     lr_decay=outer.lr_decay, tau=tau, generator=generator or gcn.generator or _rng.default_generator,
                     params=inner.model_params, samples=samples)
