"""The kNN initialisation of BASELINE config 2 against the reference's own call.

tests/golden/knn_cora.npz holds the output of the reference's knn_graph_dense
(src/data/utils.py:165-175: sklearn kneighbors_graph, k=10, cosine,
include_self=False) on the real Cora features, made by
tests/golden/make_golden.py (job knn_cora).  That fixture is the θ₀ bench.py
and the config-2 goldens use, so the sampled workload is the same on every
machine.

ldsgnn.utils.graph.knn_graph_dense (torch top-k) must pick the same neighbour
sets up to exact ties at the k-th distance: Cora's binary bag-of-words rows
tie often (≈850 rows have several neighbours at exactly the k-th cosine
distance), and sklearn's argpartition breaks such ties in an order no other
selection reproduces.  Every other entry must agree exactly."""
import numpy as np
import torch

from ldsgnn.data.planetoid import load_planetoid_npz
from ldsgnn.data.synthetic import knn_init
from ldsgnn.utils.graph import knn_graph_dense
from tests.conftest import GOLDEN


def _fixture():
    return np.load(f"{GOLDEN}/knn_cora.npz")


def test_knn_fixture_shape_and_symmetrisation():
    g = _fixture()
    n, k = 2708, int(g["k"])
    d = g["directed"]
    assert d.shape[1] == n * k and np.all(np.bincount(d[0], minlength=n) == k)  # k per row
    assert not np.any(d[0] == d[1])                                              # include_self=False
    a = np.zeros((n, n), dtype=bool)
    a[d[0], d[1]] = True
    und = a | a.T                                                                # MakeUndirected
    iu = np.triu_indices(n, 1)
    want = np.stack(iu)[:, und[iu]]
    assert np.array_equal(g["edges"], want)


def test_knn_graph_dense_matches_reference_up_to_ties():
    g = _fixture()
    data = load_planetoid_npz("cora")
    n = data.num_nodes
    got = knn_graph_dense(data.x, 10, loop=False)
    ref = torch.zeros(n, n)
    e = torch.from_numpy(g["directed"]).long()
    ref[e[0], e[1]] = 1.0
    assert torch.equal(got.sum(1), ref.sum(1))
    x = data.x.double()
    xn = x / x.norm(dim=1, keepdim=True)
    dist = 1.0 - xn @ xn.t()
    dist.fill_diagonal_(float("inf"))
    kth = torch.sort(dist, 1).values[:, 9]
    r, c = (got != ref).nonzero(as_tuple=True)
    # every disagreement is a neighbour at exactly the k-th distance (fp32 rounding of a tie)
    assert float((dist[r, c] - kth[r]).abs().max()) < 1e-6
    # so the per-row distance multisets agree
    dg = torch.sort(torch.where(got > 0, dist, torch.full_like(dist, 9.0)), 1).values[:, :10]
    dr = torch.sort(torch.where(ref > 0, dist, torch.full_like(dist, 9.0)), 1).values[:, :10]
    assert float((dg - dr).abs().max()) < 1e-6


def test_knn_init_symmetrises():
    data = load_planetoid_npz("cora")
    d = knn_init(data, k=10)
    assert torch.equal(d.dense_adj, d.dense_adj.t()) and float(d.dense_adj.diag().abs().sum()) == 0.0
