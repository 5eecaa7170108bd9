"""The BASELINE.json workloads as data (SURVEY §8(d) "Concrete inputs").

  cora           config 2 (and 4): the real Cora Planetoid split, NormalizeFeatures,
                 θ₀ = the symmetrised cosine kNN graph (k = 10) the reference's own
                 knn_graph_dense call produced (tests/golden/knn_cora.npz, made by
                 tests/golden/make_golden.py; src/data/utils.py:165-175 with
                 MakeUndirected) — identical on every machine
  cora-given     config 1: the real Cora split with its given graph (fixed adjacency)
  citeseer       config 3: the real Citeseer split, θ₀ = the given graph
  cora-synthetic a synthetic Cora-shaped problem with a torch kNN θ₀ (round-1 bench)
  synthetic20k   config 5: N = 20 000, F_in 128, X ~ U[0,1) row-normalised,
                 θ_ij ~ U(0, 1) i.i.d. (seed 20000), drawn on `device`
  synthetic20k-sparse  config 5's optional sparse variant: the same X, θ_ij ~
                 U(0, 0.01) (≈ 2·10⁶ sampled entries per graph: short rows)

Every workload returns a DenseData whose dense_adj is θ₀ (the
BernoulliGraphModel init matrix, src/models/factory.py:60-62).
"""
from __future__ import annotations

import os

import numpy as np
import torch

from ..utils.graph import DenseData
from .planetoid import FIXTURE_DIR, load_planetoid_npz
from .synthetic import knn_init, make_dataset

WORKLOADS = ("cora", "cora-given", "citeseer", "cora-synthetic", "synthetic20k", "synthetic20k-sparse")


def knn_theta0(n: int, path: str = None) -> torch.Tensor:
    """Dense 0/1 θ₀ from the committed kNN edge list (i < j pairs)."""
    z = np.load(path or os.path.join(FIXTURE_DIR, "knn_cora.npz"))
    e = torch.from_numpy(z["edges"]).long()
    a = torch.zeros(n, n)
    a[e[0], e[1]] = 1.0
    a[e[1], e[0]] = 1.0
    return a


def load_workload(name: str, seed: int = 0, device="cpu") -> DenseData:
    if name == "cora":
        data = load_planetoid_npz("cora")
        data.dense_adj = knn_theta0(data.num_nodes)
        data.name = "cora (Planetoid split), kNN theta0 (k=10, reference sklearn fixture)"
    elif name == "cora-given":
        data = load_planetoid_npz("cora")
        data.name = "cora (Planetoid split), given graph"
    elif name == "citeseer":
        data = load_planetoid_npz("citeseer")
        data.name = "citeseer (Planetoid split), given graph theta0"
    elif name == "cora-synthetic":
        data = knn_init(make_dataset("cora", seed=seed), k=10)
        data.name = "synthetic cora-shaped, torch kNN theta0"
    elif name in ("synthetic20k", "synthetic20k-sparse"):
        data = make_dataset("synthetic20k", seed=seed)
        data = data.to(device)
        g = torch.Generator(device=data.x.device).manual_seed(20000)
        data.dense_adj = torch.rand((data.num_nodes, data.num_nodes), generator=g, device=data.x.device)
        if name == "synthetic20k-sparse":
            data.dense_adj.mul_(0.01)
            data.name = "synthetic N=20000, theta ~ U(0,0.01) i.i.d. (seed 20000)"
        else:
            data.name = "synthetic N=20000, theta ~ U(0,1) i.i.d. (seed 20000)"
        return data
    else:
        raise ValueError(f"unknown workload {name!r}: one of {WORKLOADS}")
    return data.to(device)
