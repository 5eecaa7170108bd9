"""Differentiable Adam — the slice of `higher` the reference uses.

The reference's inner problem steps its GCN with
`higher.optim.DifferentiableAdam(Adam([...groups]), model.parameters())`
and `.step(loss, params=...)` (src/trainers/inner.py:6, 42-50, 71).  `higher`
(facebookresearch, unpinned git HEAD per scripts/install.sh:3-4) is neither
vendored nor installable here; this restates its published update rule:

    g   = autograd.grad(loss, params, create_graph=True)
    g  += weight_decay · p                  (per param group)
    m   = m·β1 + (1-β1)·g ;  v = v·β2 + (1-β2)·g·g
    grad of v masked to 0 where v == 0     (higher's _maybe_mask)
    p  -= (lr / (1-β1^t)) · m / (sqrt(v)/sqrt(1-β2^t) + eps)

`params`/state keep the autograd history, so a later backward differentiates
through every step back to the last `detach` — the truncated hypergradient.
"""
from __future__ import annotations

import math
from collections import defaultdict
from typing import List

import torch


class DifferentiableOptimizer:
    def __init__(self, other: torch.optim.Optimizer, reference_params, track_higher_grads: bool = True):
        reference_params = list(reference_params)
        self.param_groups = []
        self._group_to_param_list: List[List[int]] = []
        for group in other.param_groups:
            g = {k: v for k, v in group.items() if k != "params"}
            mapping = []
            for p in group["params"]:
                idx = [i for i, rp in enumerate(reference_params) if rp is p]
                if not idx:
                    raise ValueError("optimizer parameter not among reference_params")
                mapping.append(idx[0])
            g["params"] = [reference_params[i] for i in mapping]
            self.param_groups.append(g)
            self._group_to_param_list.append(mapping)
        # state: per group, per param index in group -> dict
        self.state = [defaultdict(dict) for _ in self.param_groups]
        self._track_higher_grads = track_higher_grads

    def step(self, loss: torch.Tensor, params=None, **kwargs):
        params = list(params)
        grad_targets = [p if p.requires_grad else torch.tensor([], requires_grad=True) for p in params]
        all_grads = torch.autograd.grad(loss, grad_targets, create_graph=self._track_higher_grads,
                                        allow_unused=True)
        grouped = []
        for group, mapping in zip(self.param_groups, self._group_to_param_list):
            grads = []
            for i, index in enumerate(mapping):
                group["params"][i] = params[index]
                grads.append(all_grads[index])
            grouped.append(grads)
        self._update(grouped)
        new_params = params[:]
        for group, mapping in zip(self.param_groups, self._group_to_param_list):
            for p, index in zip(group["params"], mapping):
                new_params[index] = p if self._track_higher_grads else p.detach().requires_grad_()
        return new_params

    def _update(self, grouped_grads):
        raise NotImplementedError

    def truncate(self) -> None:
        """Cut the autograd history held by the optimizer, in place: every
        tensor in the state (m, v) and among the group hyper-parameters
        becomes a leaf that requires grad.  Plain numbers (step, lr) and the
        group's params list are left alone.  This is what the reference's
        InnerProblemTrainer.detach_optimizer does to higher's state
        (src/trainers/inner.py:110-125)."""
        tensors = [value for group in self.param_groups for value in group.values()]
        tensors += [value for per_group in self.state for slot in per_group.values() for value in slot.values()]
        for t in tensors:
            if isinstance(t, torch.Tensor):
                t.detach_().requires_grad_()


def _maybe_mask(tensor: torch.Tensor, mask: torch.Tensor) -> None:
    if isinstance(tensor, torch.Tensor) and tensor.requires_grad:
        tensor.register_hook(lambda grad: grad.masked_fill(mask, 0.0))


class DifferentiableAdam(DifferentiableOptimizer):
    def _update(self, grouped_grads):
        for group_idx, (group, grads) in enumerate(zip(self.param_groups, grouped_grads)):
            beta1, beta2 = group["betas"]
            weight_decay = group["weight_decay"]
            for p_idx, (p, g) in enumerate(zip(group["params"], grads)):
                if g is None:
                    continue
                state = self.state[group_idx][p_idx]
                if len(state) == 0:
                    state["step"] = 0
                    state["exp_avg"] = torch.zeros_like(p.data)
                    state["exp_avg_sq"] = torch.zeros_like(p.data)
                exp_avg, exp_avg_sq = state["exp_avg"], state["exp_avg_sq"]
                state["step"] += 1
                bias_correction1 = 1 - beta1 ** state["step"]
                bias_correction2 = 1 - beta2 ** state["step"]
                if weight_decay != 0:
                    g = g + (weight_decay * p)
                state["exp_avg"] = exp_avg = (exp_avg * beta1) + (1 - beta1) * g
                state["exp_avg_sq"] = exp_avg_sq = (exp_avg_sq * beta2) + (1 - beta2) * g * g
                mask = exp_avg_sq == 0.0
                _maybe_mask(exp_avg_sq, mask)
                denom = (exp_avg_sq.sqrt() / math.sqrt(bias_correction2)) + group["eps"]
                step_size = group["lr"] / bias_correction1
                group["params"][p_idx] = torch.addcdiv(p, exp_avg, denom, value=-step_size)
