"""Synthetic datasets of the BASELINE.json configs' shapes.

Cora-shaped: N=2708, F_in=1433, C=7, ~1.27 % non-zero binary features
(row-normalised like torch_geometric's NormalizeFeatures), Planetoid split
sizes 140/500/1000 (src/data/dataloader.py:19-29 defaults).  Citeseer-shaped:
3327/3703/6.  Synthetic N=20000, F_in=128, X ~ U[0,1) row-normalised, C=7
(SURVEY §8(d) config 5).  Labels carry a weak feature signal so training
curves are meaningful; no real data is implied.
"""
from __future__ import annotations

import torch

from ..utils.graph import DenseData, knn_graph_dense

SHAPES = {
    "cora": dict(n=2708, f_in=1433, classes=7, density=0.0127, edges=5278),
    "citeseer": dict(n=3327, f_in=3703, classes=6, density=0.0086, edges=4552),
    "synthetic20k": dict(n=20000, f_in=128, classes=7, density=1.0, edges=0),
}


def make_dataset(name: str = "cora", seed: int = 0, device="cpu", n_train: int = 140,
                 n_val: int = 500, n_test: int = 1000) -> DenseData:
    sh = SHAPES[name]
    n, f_in, c = sh["n"], sh["f_in"], sh["classes"]
    g = torch.Generator().manual_seed(seed)
    y = torch.randint(0, c, (n,), generator=g)
    if sh["density"] < 1.0:
        x = (torch.rand(n, f_in, generator=g) < sh["density"]).float()
        # class signal: each class prefers a block of features
        block = f_in // c
        bonus = torch.rand(n, block, generator=g) < 4 * sh["density"]
        for k in range(c):
            rows = (y == k).nonzero().squeeze(1)
            x[rows, k * block:(k + 1) * block] = torch.maximum(
                x[rows, k * block:(k + 1) * block], bonus[rows].float())
    else:
        x = torch.rand(n, f_in, generator=g)
    x = x / x.sum(1, keepdim=True).clamp(min=1.0e-12)  # NormalizeFeatures
    # given graph: homophilous random edges
    adj = torch.zeros(n, n)
    if sh["edges"]:
        src = torch.randint(0, n, (4 * sh["edges"],), generator=g)
        dst = torch.randint(0, n, (4 * sh["edges"],), generator=g)
        same = (y[src] == y[dst]) | (torch.rand(src.numel(), generator=g) < 0.2)
        src, dst = src[same][: sh["edges"]], dst[same][: sh["edges"]]
        adj[src, dst] = 1.0
        adj[dst, src] = 1.0
        adj.fill_diagonal_(0.0)
    perm = torch.randperm(n, generator=g)
    masks = []
    start = 0
    for size in (n_train, n_val, n_test):
        m = torch.zeros(n, dtype=torch.bool)
        m[perm[start:start + size]] = True
        masks.append(m)
        start += size
    data = DenseData(x=x, y=y, dense_adj=adj, train_mask=masks[0], val_mask=masks[1],
                     test_mask=masks[2], num_classes=c, name=f"{name}-synthetic")
    return data.to(device)


def knn_init(data: DenseData, k: int = 10) -> DenseData:
    """KNNGraph + MakeUndirected (src/data/transforms.py:15-37): θ₀ graph."""
    a = knn_graph_dense(data.x, k, loop=False)
    data.dense_adj = torch.maximum(a, a.t())
    return data
