"""Inner problem of the bilevel loop: the GCN trained by a differentiable Adam
(reference API: src/trainers/inner.py:15-125).

Behaviour kept from the reference:
- `train_step(graph, mask)` runs the GCN in train mode (dropout on), takes the
  NLL over `mask` (default: the train mask) and one differentiable Adam step;
  the new weights keep their autograd history (create_graph), so a later
  backward reaches θ through every step since the last `detach()`;
- Adam has two groups: layer_in with weight decay, layer_out without
  (src/trainers/inner.py:42-50); its step counter survives `detach()` and
  restarts only in `reset_optimizer()`;
- `detach()` is the truncation point: weights and optimizer state become
  fresh leaves.
Difference: a mask argument is tested with `is None`, not truthiness (the
reference's `mask or …` raises for a multi-element tensor).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, Iterable, Optional

import torch
import torch.nn.functional as F
from torch.optim import Adam

from ..models.gcn import MetaDenseGCN
from ..optim import DifferentiableAdam, DifferentiableOptimizer
from ..utils.evaluation import accuracy
from ..utils.graph import is_square_matrix
from . import Metrics


def copy_detach_parameter_dict(parameters: OrderedDict) -> OrderedDict:
    """A new dict (same key order) whose values are detached copies that
    require grad (src/trainers/inner.py:15-19)."""
    return OrderedDict((name, t.detach().clone().requires_grad_(True)) for name, t in parameters.items())


class InnerProblemTrainer:
    def __init__(self, model: MetaDenseGCN, data, lr: float = 0.01, weight_decay: float = 1e-4):
        self.model = model
        self.data = data
        self.lr = lr
        self.weight_decay = weight_decay
        self.optimizer: Optional[DifferentiableOptimizer] = None
        self.model_params: OrderedDict = OrderedDict(model.named_parameters())
        self.reset_optimizer()

    # -- weights and optimizer -------------------------------------------------
    def reset_weights(self):
        self.model.reset_weights()
        self.model_params = OrderedDict(self.model.named_parameters())

    def reset_optimizer(self) -> None:
        groups = [dict(params=list(self.model.layer_in.parameters()), weight_decay=self.weight_decay),
                  dict(params=list(self.model.layer_out.parameters()))]
        self.optimizer = DifferentiableAdam(Adam(groups, lr=self.lr), self.model.parameters())

    def copy_model_params(self) -> Dict:
        return copy_detach_parameter_dict(self.model_params)

    def _set_params(self, values: Iterable[torch.Tensor]) -> None:
        self.model_params = OrderedDict(zip(self.model_params.keys(), values))

    # -- steps ----------------------------------------------------------------
    def _nll_and_accuracy(self, predictions: torch.Tensor, mask: torch.Tensor):
        logits, labels = predictions[mask], self.data.y[mask]
        return F.nll_loss(logits, labels), accuracy(logits, labels)

    def model_forward(self, graph, is_train: bool = True) -> torch.Tensor:
        self.model.train(mode=is_train)
        return self.model(self.data.x, graph, params=self.model_params)

    def train_step(self, graph, mask: torch.Tensor = None) -> Metrics:
        assert is_square_matrix(graph)
        loss, acc = self._nll_and_accuracy(self.model_forward(graph, is_train=True),
                                           self.data.train_mask if mask is None else mask)
        self._set_params(self.optimizer.step(loss, params=self.model_params.values()))
        return Metrics(loss=loss.item(), acc=acc)

    def evaluate(self, graph, mask: torch.Tensor = None) -> Metrics:
        self.model.eval()
        with torch.no_grad():
            loss, acc = self._nll_and_accuracy(self.model_forward(graph, is_train=False),
                                               self.data.val_mask if mask is None else mask)
        return Metrics(loss=loss.item(), acc=acc)

    # -- truncation -----------------------------------------------------------
    def detach(self) -> None:
        self.model_params = copy_detach_parameter_dict(self.model_params)
        self.detach_optimizer()

    def detach_optimizer(self) -> None:
        self.optimizer.truncate()
