"""Graph utilities with the reference's names and semantics (src/utils/graph.py).

The dense helpers (`to_undirected`, `triu_values_to_symmetric_matrix`,
`normalize_adjacency_matrix`, ...) keep the reference's dense semantics for
API parity and inspection; the hot path never calls them — it samples,
normalises and aggregates through ldsgnn.ops (HIP kernels) without forming an
N×N matrix.
"""
from __future__ import annotations

from math import sqrt
from typing import Tuple, Union

import numpy as np
import torch


class DenseData:
    """Container with the fields the trainers read (src/utils/graph.py:15-24):
    x, y, dense_adj, train_mask, val_mask, test_mask, num_classes, name.
    `graph` optionally holds the hot-path CSR form of dense_adj."""

    def __init__(self, **kwargs):
        self.x = None
        self.y = None
        self.dense_adj: torch.Tensor = None
        self.train_mask: torch.Tensor = None
        self.val_mask: torch.Tensor = None
        self.test_mask: torch.Tensor = None
        self.num_classes: int = -1
        self.name: str = ""
        self.graph = None
        for k, v in kwargs.items():
            setattr(self, k, v)

    @property
    def num_nodes(self) -> int:
        return int(self.x.size(0))

    @property
    def num_features(self) -> int:
        return int(self.x.size(1))

    def to(self, device) -> "DenseData":
        out = DenseData()
        for k, v in self.__dict__.items():
            setattr(out, k, v.to(device) if isinstance(v, torch.Tensor) else v)
        return out


def is_square_matrix(tensor) -> bool:
    """src/utils/graph.py:119-120; also true for hot-path graphs."""
    return len(tensor.size()) == 2 and tensor.size(0) == tensor.size(1)


def to_undirected(adj: torch.Tensor, from_triu_only: bool = False) -> torch.Tensor:
    """src/utils/graph.py:27-38"""
    assert is_square_matrix(adj)
    if not from_triu_only:
        return torch.max(adj, adj.t())
    triu = adj.triu(1)
    return triu + triu.t() + torch.diag(adj.diag())


def get_triu_values(adj: torch.Tensor) -> torch.Tensor:
    """src/utils/graph.py:41-45 — row-major upper triangle incl. the diagonal."""
    assert adj.size(0) == adj.size(1)
    n = adj.size(0)
    idx = torch.triu_indices(n, n, device=adj.device)
    return adj[idx[0], idx[1]]


def split_mask(mask: torch.Tensor, ratio: float = 0.5, shuffle: bool = True,
               device: Union[str, torch.device] = "cpu") -> Tuple[torch.Tensor, torch.Tensor]:
    """src/utils/graph.py:48-76 (numpy global RNG for the shuffle, as there)."""
    nonzero_indices = mask.nonzero()
    if shuffle:
        shuffled = np.arange(nonzero_indices.size(0))
        np.random.shuffle(shuffled)
        nonzero_indices = nonzero_indices[torch.as_tensor(shuffled, device=nonzero_indices.device)]
    split_index = int(nonzero_indices.size(0) * ratio)
    first_mask = torch.zeros_like(mask, dtype=torch.bool, device=device)
    first_mask[nonzero_indices[:split_index]] = 1
    second_mask = torch.zeros_like(mask, dtype=torch.bool, device=device)
    second_mask[nonzero_indices[split_index:]] = 1
    return first_mask, second_mask


def add_self_loops(adj: torch.Tensor) -> torch.Tensor:
    """src/utils/graph.py:123-133 — clone, diagonal SET to 1."""
    assert is_square_matrix(adj)
    c = adj.clone()
    c.fill_diagonal_(1.0)
    return c


def normalize_adjacency_matrix(dense_adj: torch.Tensor) -> torch.Tensor:
    """src/utils/graph.py:136-153 (dense reference semantics)."""
    assert is_square_matrix(dense_adj)
    a = add_self_loops(dense_adj)
    inv_sqrt = 1.0 / a.sum(dim=1).sqrt()
    d = torch.diag(inv_sqrt).to(dense_adj.device)
    return d @ a @ d


def triu_values_to_symmetric_matrix(triu_values: torch.Tensor) -> torch.Tensor:
    """src/utils/graph.py:166-181 (dense; the hot path never forms it)."""
    assert len(triu_values.size()) == 1
    n = num_nodes_from_triu_shape(triu_values.size(0))
    idx = torch.triu_indices(n, n, device=triu_values.device)
    adj = torch.zeros((n, n), device=triu_values.device, dtype=triu_values.dtype)
    adj[idx[0], idx[1]] = triu_values
    adj = to_undirected(adj, from_triu_only=True)
    return adj.clamp(0.0, 1.0)


def num_nodes_from_triu_shape(n_triu_values: int) -> int:
    """src/utils/graph.py:184-192 (same arithmetic)."""
    return int(0.5 * sqrt((8 * n_triu_values + 1) - 1))


def cosine_similarity(a: torch.Tensor, b: torch.Tensor = None, eps: float = 1e-8) -> torch.Tensor:
    """src/utils/graph.py:156-163"""
    a_norm = a.norm(p=2, dim=1, keepdim=True)
    if b is None:
        b, b_norm = a, a_norm
    else:
        b_norm = b.norm(p=2, dim=1, keepdim=True)
    return (torch.mm(a, b.t()) / (a_norm * b_norm.t()).clamp(min=eps)).clamp_max(1.0)


def knn_graph_dense(x: torch.Tensor, k: int, loop: bool = True, metric: str = "cosine") -> torch.Tensor:
    """src/data/utils.py:165-175: sklearn's kneighbors_graph(mode='connectivity',
    include_self=loop) as a dense 0/1 matrix, directed rows (row i marks its k
    nearest), on x's device.  metric "cosine": distance 1 - cos; "dot" (the
    reference passes np.dot as a callable metric, so sklearn treats the dot
    product as a distance): the smallest dot products are the nearest.

    sklearn's rule for the query point itself:
    - include_self=True: the k nearest of all points — the point itself only
      if its own distance ranks (for cosine it always does: distance 0);
    - include_self=False: the k + 1 nearest are taken and the point itself is
      dropped from them; when it is not among them, the FIRST (nearest)
      candidate is dropped instead (sklearn.neighbors KNeighborsMixin
      .kneighbors with X=None).  Under "dot" a point's own distance |x|² is
      rarely among the smallest, so its nearest neighbour is skipped.
    Cosine is pinned against the reference's own sklearn calls
    (tests/golden/knn_cora.npz, graph_models.npz knn_cosine_).  "dot" is NOT
    drop-in with the reference: the reference hands np.dot to sklearn as a
    callable metric, for which sklearn's default search is a BallTree whose
    pruning assumes a metric (dot "distances" are negative), so its pattern
    depends on the tree.  This function computes the exact k nearest under
    the same dissimilarity instead — the reference's call with
    algorithm="brute", a modified reference call (golden knn_dotbrute_,
    bit-exact).  Against the reference's own dot golden (knn_dot_, 70 nodes,
    k = 7) the sampled graph differs in 126 of 4,900 entries
    (tests/test_graph_models_cpu.py::test_knn_dot_distance_from_reference_balltree)."""
    x = x.detach().float()
    n = x.size(0)
    if metric == "cosine":   # nearest = largest cosine; a point is its own nearest (distance 0)
        xn = x / x.norm(dim=1, keepdim=True).clamp(min=1e-12)
        score = xn @ xn.t()
        score.fill_diagonal_(float("inf") if loop else -float("inf"))
        idx = torch.topk(score, k, dim=1).indices
    elif metric == "dot":    # nearest = smallest dot product
        score = -(x @ x.t())
        if loop:
            idx = torch.topk(score, k, dim=1).indices
        else:
            cand = torch.topk(score, k + 1, dim=1).indices            # nearest first
            rows = torch.arange(n, device=x.device).unsqueeze(1)
            is_self = cand == rows
            drop = torch.where(is_self.any(1, keepdim=True), is_self,
                               torch.arange(k + 1, device=x.device).unsqueeze(0) == 0)
            idx = cand[~drop].view(n, k)
    else:
        raise NotImplementedError(f"knn metric {metric}")
    a = torch.zeros((n, n), dtype=torch.float32, device=x.device)
    a.scatter_(1, idx, 1.0)
    return a

