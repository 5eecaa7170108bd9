"""θ pre-training of the LDS Bernoulli model (src/trainers/pretrainer.py:18-143).

OuterProblemTrainer(pretrain=True) (the reference's outer-trainer default,
src/trainers/outer.py:54-55,107-109,125) fits P = triu_values_to_symmetric_matrix(θ)
to the training edges before the bilevel loop: weighted BCE against the dense
training adjacency (positive weight = #non-edges / #edges), Adam (lr 0.01),
early stopping on the validation edges' average precision (patience 20, at most
400 epochs), then the test edges' AUC / AP.

Here one epoch is ONE fused HIP launch over the packed θ (lds_pretrain_step:
P, BCE gradient, clamp / symmetrisation backward, Adam) — the reference's
dense N×N P, weight matrix and gradient are never formed.  The edge split is
torch_geometric 1.3.2's GAE.split_edges (restated, the library is absent):
upper-triangle edges shuffled, 5 % validation / 10 % test positives, as many
negatives drawn from the non-edges, training positives made undirected.  Its
shuffles use a seeded torch.Generator instead of the global torch / `random`
streams, so splits are reproducible but not the reference's draws.

Quirk kept: the reference's EarlyStopping stores model.state_dict() — views of
the live θ — so loading the "best" state at the end is a no-op and pre-training
ends with the last θ (src/utils/early_stopping.py:27-30 + pretrainer.py:56).
"""
from __future__ import annotations

import math
from typing import Dict, Optional

import numpy as np
import torch

from .. import _native as nat
from ..utils.early_stopping import EarlyStopping


def split_edges(dense_adj: torch.Tensor, val_ratio: float = 0.05, test_ratio: float = 0.1,
                generator: Optional[torch.Generator] = None) -> Dict[str, torch.Tensor]:
    """GAE.split_edges (torch_geometric 1.3.2) on a dense symmetric adjacency;
    returns 2 × E index tensors (CPU, int64)."""
    adj = dense_adj.detach().cpu()
    n = adj.size(0)
    row, col = torch.triu(adj, diagonal=1).nonzero(as_tuple=True)  # edge_index order, row < col
    n_v = int(math.floor(val_ratio * row.numel()))
    n_t = int(math.floor(test_ratio * row.numel()))
    perm = torch.randperm(row.numel(), generator=generator)
    row, col = row[perm], col[perm]
    out = {"val_pos": torch.stack([row[:n_v], col[:n_v]]),
           "test_pos": torch.stack([row[n_v:n_v + n_t], col[n_v:n_v + n_t]])}
    r, c = row[n_v + n_t:], col[n_v + n_t:]
    out["train_pos"] = torch.stack([torch.cat([r, c]), torch.cat([c, r])])  # to_undirected
    neg = torch.ones(n, n, dtype=torch.bool).triu(diagonal=1)
    neg[row, col] = False
    neg_row, neg_col = neg.nonzero(as_tuple=True)
    pick = torch.randperm(neg_row.numel(), generator=generator)[: min(n_v + n_t, neg_row.numel())]
    neg_row, neg_col = neg_row[pick], neg_col[pick]
    out["val_neg"] = torch.stack([neg_row[:n_v], neg_col[:n_v]])
    out["test_neg"] = torch.stack([neg_row[n_v:n_v + n_t], neg_col[n_v:n_v + n_t]])
    return out


def edges_to_bits(edge_index: torch.Tensor, n: int, device) -> torch.Tensor:
    """n × words uint64 (as int64) bitmask of a directed edge list."""
    words = nat.lib.lds_bitmask_words(n)
    bits = np.zeros((n, words * 64), dtype=bool)
    e = edge_index.cpu().numpy()
    bits[e[0], e[1]] = True
    packed = np.packbits(bits.reshape(n, words, 64)[:, :, ::-1], axis=-1)  # bit j%64 of word j/64
    words64 = packed.view(">u8").reshape(n, words).astype(np.uint64)
    return torch.from_numpy(words64.view(np.int64)).to(device)


class Pretrainer:
    """src/trainers/pretrainer.py:18-113 for BernoulliGraphModel (undirected)."""

    def __init__(self, model, data, lr: float = 0.01, optimizer: str = "adam", patience: int = 20,
                 max_epochs: int = 400, generator: Optional[torch.Generator] = None,
                 betas=(0.9, 0.999), eps: float = 1e-8, split: Optional[Dict[str, torch.Tensor]] = None):
        """`split`: a precomputed edge split (split_edges' keys) instead of
        drawing one from data.dense_adj — the reference's split is a
        torch_geometric draw this repository cannot reproduce, so the golden
        test hands both sides the same split."""
        assert optimizer.lower() in ["sgd", "adam"]
        if optimizer.lower() != "adam" or getattr(model, "directed", False):
            raise NotImplementedError("fused pre-training implements Adam on the undirected Bernoulli model")
        self.model = model
        theta = model.probs
        nat.require_device(theta, "Pretrainer")
        self.n = n = model.num_nodes
        self.lr, self.betas, self.eps = float(lr), betas, float(eps)
        self.split = dict(split) if split is not None else split_edges(data.dense_adj, generator=generator)
        self.train_bits = edges_to_bits(self.split["train_pos"], n, theta.device)
        t_sum = float(self.split["train_pos"].size(1))
        self.pos_weight = float(np.float32((n * n - t_sum) / t_sum))  # (numel - sum) / sum
        self.m = torch.zeros_like(theta.data)
        self.v = torch.zeros_like(theta.data)
        self.step = 0
        self.loss_rows = torch.zeros(n, dtype=torch.float32, device=theta.device)
        self.early_stopper = EarlyStopping(patience=patience, max_epochs=max_epochs)
        self.history = []

    def train(self) -> Dict[str, float]:
        epoch = 0
        while not self.early_stopper.abort:
            self.train_step(epoch)
            epoch += 1
        self.model.load_state_dict(self.early_stopper.best_model_state_dict())
        return self.evaluate(self.split["test_pos"], self.split["test_neg"])

    def train_step(self, epoch: int) -> float:
        self.model.train()
        self.step += 1
        theta = self.model.probs.data
        nat.call("lds_pretrain_step", nat.ptr(theta), self.n, nat.ptr(self.train_bits), self.train_bits.size(1),
                 self.pos_weight, nat.ptr(self.m), nat.ptr(self.v), self.step, self.lr, self.betas[0],
                 self.betas[1], self.eps, nat.ptr(self.loss_rows), nat.stream_of(theta.device))
        val = self.evaluate(self.split["val_pos"], self.split["val_neg"])
        loss = float(self.loss_rows.double().sum().item()) / (self.n * self.n)
        self.history.append(dict(epoch=epoch, loss=loss, **{f"val_{k}": v for k, v in val.items()}))
        self.early_stopper.update(-val.get("average_precision", 0.0), model=self.model)
        return loss

    def edge_probabilities(self, index: torch.Tensor) -> torch.Tensor:
        """P at (i, j) pairs without forming P: clamp(θ[tri(min, max)], 0, 1)."""
        n = self.n
        i = torch.minimum(index[0], index[1]).long()
        j = torch.maximum(index[0], index[1]).long()
        tri = i * (2 * n - i + 1) // 2 + (j - i)
        return self.model.probs.detach()[tri.to(self.model.probs.device)].clamp(0.0, 1.0)

    def evaluate(self, pos_index: torch.Tensor, neg_index: torch.Tensor) -> Dict[str, float]:
        from sklearn.metrics import average_precision_score, roc_auc_score
        self.model.eval()
        with torch.no_grad():
            pred = torch.cat([self.edge_probabilities(pos_index), self.edge_probabilities(neg_index)]).cpu()
        y = torch.cat([torch.ones(pos_index.size(1)), torch.zeros(neg_index.size(1))])
        return {"auc": float(roc_auc_score(y, pred)), "average_precision": float(average_precision_score(y, pred))}
