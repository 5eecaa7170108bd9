"""Metrics and the S-sample empirical evaluation (src/utils/evaluation.py)."""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict, Tuple

import numpy as np
import torch
from torch.nn import functional as F

from ..trainers import Metrics


def accuracy(predictions: torch.Tensor, labels: torch.Tensor) -> float:
    """src/utils/evaluation.py:15-22"""
    return (torch.argmax(predictions, dim=-1) == labels).float().mean().item()


def evaluate(model: torch.nn.Module, data, adj_matrix=None) -> Dict:
    """src/utils/evaluation.py:25-48; `adj_matrix` may be a hot-path graph."""
    model.eval()
    with torch.no_grad():
        graph = adj_matrix if adj_matrix is not None else (
            data.graph if getattr(data, "graph", None) is not None else data.dense_adj)
        out = model(data.x, graph)
        val_acc = accuracy(out[data.val_mask], data.y[data.val_mask])
        val_loss = F.nll_loss(out[data.val_mask], data.y[data.val_mask]).item()
        test_acc = accuracy(out[data.test_mask], data.y[data.test_mask])
        test_loss = F.nll_loss(out[data.test_mask], data.y[data.test_mask]).item()
    return {"val.accuracy": val_acc, "val.loss": val_loss,
            "test.accuracy": test_acc, "test.loss": test_loss}


def empirical_mean_loss(gcn, graph_model, n_samples: int, data,
                        model_parameters: OrderedDict = None) -> Tuple[Metrics, Metrics]:
    """src/utils/evaluation.py:51-84: mean NLL/accuracy over `n_samples` graphs
    drawn from the graph model, no grad.  Losses stay on device and are reduced
    once (one host sync instead of 4·S)."""
    gcn.eval()
    graph_model.eval()
    with torch.no_grad():
        vals = []
        for _ in range(n_samples):
            graph = graph_model.sample()
            pred = gcn(data.x, graph, params=model_parameters)
            vm, tm = data.val_mask, data.test_mask
            vals.append(torch.stack([
                F.nll_loss(pred[vm], data.y[vm]),
                (torch.argmax(pred[vm], dim=-1) == data.y[vm]).float().mean(),
                F.nll_loss(pred[tm], data.y[tm]),
                (torch.argmax(pred[tm], dim=-1) == data.y[tm]).float().mean(),
            ]))
        host = torch.stack(vals).double().cpu().numpy()
    val_metrics = Metrics(loss=np.mean(host[:, 0]).item(), acc=np.mean(host[:, 1]).item())
    test_metrics = Metrics(loss=np.mean(host[:, 2]).item(), acc=np.mean(host[:, 3]).item())
    return val_metrics, test_metrics
