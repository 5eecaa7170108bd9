"""Inner problem: GCN training with a differentiable optimizer
(src/trainers/inner.py:15-125), same API and truncation semantics."""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, List

import torch
import torch.nn.functional as F
from torch.optim import Adam

from ..models.gcn import MetaDenseGCN
from ..optim import DifferentiableAdam, DifferentiableOptimizer
from ..utils.evaluation import accuracy
from ..utils.graph import is_square_matrix
from . import Metrics


def copy_detach_parameter_dict(parameters: OrderedDict) -> OrderedDict:
    """src/trainers/inner.py:15-19"""
    d = parameters.copy()
    for key in d.keys():
        d[key] = d[key].detach().clone().requires_grad_(True)
    return d


class InnerProblemTrainer:
    def __init__(self, model: MetaDenseGCN, data, lr: float = 0.01, weight_decay: float = 1e-4):
        self.model = model
        self.lr = lr
        self.weight_decay = weight_decay
        self.model_params: OrderedDict = OrderedDict(model.named_parameters())
        self.optimizer: DifferentiableOptimizer = None
        self.data = data
        self.reset_optimizer()

    def reset_weights(self):
        self.model.reset_weights()
        self.model_params = OrderedDict(self.model.named_parameters())

    def reset_optimizer(self) -> None:
        """Group 0 (layer_in) has weight decay, group 1 (layer_out) none
        (src/trainers/inner.py:42-50)."""
        optimizer = Adam([
            {"params": self.model.layer_in.parameters(), "weight_decay": self.weight_decay},
            {"params": self.model.layer_out.parameters()},
        ], lr=self.lr)
        self.optimizer = DifferentiableAdam(optimizer, self.model.parameters())

    def copy_model_params(self) -> Dict:
        return copy_detach_parameter_dict(self.model_params)

    def train_step(self, graph, mask: torch.Tensor = None) -> Metrics:
        """src/trainers/inner.py:55-74"""
        assert is_square_matrix(graph)
        predictions = self.model_forward(graph, is_train=True)
        mask = mask if mask is not None else self.data.train_mask
        loss = F.nll_loss(predictions[mask], self.data.y[mask])
        acc = accuracy(predictions[mask], self.data.y[mask])
        new_model_params = self.optimizer.step(loss, params=self.model_params.values())
        self._update_model_params(list(new_model_params))
        return Metrics(loss=loss.item(), acc=acc)

    def model_forward(self, graph, is_train: bool = True) -> torch.Tensor:
        self.model.train(mode=is_train)
        return self.model(self.data.x, graph, params=self.model_params)

    def evaluate(self, graph, mask: torch.Tensor = None) -> Metrics:
        self.model.eval()
        with torch.no_grad():
            predictions = self.model_forward(graph, is_train=False)
            mask = mask if mask is not None else self.data.val_mask
            loss = F.nll_loss(predictions[mask], self.data.y[mask])
            acc = accuracy(predictions[mask], self.data.y[mask])
        return Metrics(loss=loss.item(), acc=acc)

    def detach(self) -> None:
        """Truncation point (src/trainers/inner.py:98-104)."""
        self.model_params = copy_detach_parameter_dict(self.model_params)
        self.detach_optimizer()

    def _update_model_params(self, new_model_params: List[torch.Tensor]) -> None:
        for i, name in enumerate(self.model_params.keys()):
            self.model_params[name] = new_model_params[i]

    def detach_optimizer(self):
        """src/trainers/inner.py:110-125: state tensors become fresh leaves."""
        for group in self.optimizer.param_groups:
            for k, v in group.items():
                if isinstance(v, torch.Tensor):
                    v.detach_().requires_grad_()
        for state_dict in self.optimizer.state:
            for k, v_dict in state_dict.items():
                for k2, v2 in v_dict.items():
                    if isinstance(v2, torch.Tensor):
                        v2.detach_().requires_grad_()
