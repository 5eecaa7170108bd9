"""Host-side pieces of the embedding / GAE graph models
that need no GPU: the kNN pattern with the reference's metrics, the dense
sparsification semantics, the factory's error behaviour."""
import os

import numpy as np
import pytest
import torch

from ldsgnn.models.factory import GraphGenerativeModelFactory
from ldsgnn.models.sampling import SPARSIFICATION, sparsify
from ldsgnn.utils.graph import DenseData, knn_graph_dense

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_knn_dot_metric_is_a_distance():
    """np.dot passed to sklearn as a metric is read as a distance
    (src/models/sampling.py:30-32, src/data/utils.py:165-175).  Without
    include_self sklearn takes the k + 1 nearest and drops the query point —
    or, when the point is not among them (its own "distance" |x|² is large),
    the nearest one: row 0's dots with rows 0..3 are 1, 2, -1, 0, so the two
    nearest are rows 2 and 3, row 0 is not among them, row 2 is dropped."""
    x = torch.tensor([[1.0, 0.0], [2.0, 0.0], [-1.0, 0.0], [0.0, 1.0]])
    a = knn_graph_dense(x, 1, loop=False, metric="dot")
    assert torch.equal(a[0], torch.tensor([0.0, 0.0, 0.0, 1.0]))
    c = knn_graph_dense(x, 1, loop=False, metric="cosine")
    assert torch.equal(c[0], torch.tensor([0.0, 1.0, 0.0, 0.0]))


@pytest.mark.parametrize("loop", [False, True])
@pytest.mark.parametrize("metric", ["dot", "cosine"])
def test_knn_matches_sklearn_brute_force(loop, metric):
    """The same pattern as sklearn's exact search (algorithm="brute") with the
    reference's metric arguments, on random embeddings."""
    import numpy as np
    from sklearn.neighbors import NearestNeighbors
    g = torch.Generator().manual_seed(3)
    x = torch.randn(60, 6, generator=g)
    nn = NearestNeighbors(n_neighbors=5, metric=np.dot if metric == "dot" else metric, algorithm="brute")
    nn.fit(x.numpy())
    ref = nn.kneighbors_graph(x.numpy() if loop else None, n_neighbors=5, mode="connectivity").toarray()
    assert np.array_equal(knn_graph_dense(x, 5, loop=loop, metric=metric).numpy(), ref)


def test_knn_loop_includes_self_first():
    """include_self=True (the reference's default, src/data/utils.py:165-175)."""
    g = torch.Generator().manual_seed(0)
    x = torch.randn(20, 5, generator=g)
    a = knn_graph_dense(x, 3, loop=True)
    assert torch.equal(a.diagonal(), torch.ones(20)) and torch.equal(a.sum(1), torch.full((20,), 3.0))
    b = knn_graph_dense(x, 3, loop=False)
    assert torch.equal(b.diagonal(), torch.zeros(20))


def test_dense_sparsify_eps_and_knn_on_cpu():
    g = torch.Generator().manual_seed(1)
    p = torch.rand(12, 12, generator=g, requires_grad=True)
    out = sparsify(p, SPARSIFICATION.EPS, eps=0.4)
    assert torch.equal(out.detach(), torch.where(p.detach() < 0.4, torch.zeros(()), p.detach()))
    out.sum().backward()
    assert torch.equal(p.grad, (p.detach() >= 0.4).float())
    emb = torch.randn(12, 3, generator=g)
    kn = sparsify(p.detach(), SPARSIFICATION.KNN, embeddings=emb, k=4)
    assert torch.equal((kn != 0).float(), knn_graph_dense(emb, 4, loop=False) * (p.detach() != 0).float())
    with pytest.raises(AssertionError):
        sparsify(p.detach(), SPARSIFICATION.KNN, embeddings=None, k=4)
    with pytest.raises(AssertionError):
        sparsify(p.detach(), SPARSIFICATION.KNN, embeddings=emb, k=12)
    with pytest.raises(AssertionError):
        sparsify(p.detach(), SPARSIFICATION.EPS, eps=None)


def test_factory_unknown_model_and_optimizer():
    data = DenseData(x=torch.zeros(3, 2), dense_adj=torch.zeros(3, 3))
    fac = GraphGenerativeModelFactory(data)
    with pytest.raises(NotImplementedError):
        fac.create("vgae")
    with pytest.raises(NotImplementedError):
        fac.optimizer(torch.nn.Linear(2, 2))
    with pytest.raises(NotImplementedError):
        GraphGenerativeModelFactory.get_optimizer("rmsprop")


def test_knn_dot_distance_from_reference_balltree():
    """knn_metric="dot" is the exact k nearest under -x·y (the reference's
    call with sklearn's brute-force search), not the reference's own BallTree
    pattern.  On the reference goldens' 70 embeddings (k = 7,
    include_self=False) with the goldens' uniforms: bit-exact against
    knn_dotbrute_ (the reference code with algorithm="brute"), and the
    recorded distance from the reference's default call (knn_dot_): 126 of
    the 4,900 sampled entries differ (100 edges here, 122 there)."""
    g = np.load(os.path.join(ROOT, "tests", "golden", "graph_models.npz"))
    e = torch.from_numpy(g["emb_e"])
    p = torch.sigmoid(e @ e.t())
    knn = knn_graph_dense(e, 7, loop=False, metric="dot")

    def sample(key):  # src/models/sampling.py:19-36, 47-79 on the CPU: knn mask, triu draw, symmetric
        a = torch.triu(torch.from_numpy(g[key + "u"]) < p * knn, 1)
        return (a | a.t()).float()
    assert torch.equal(sample("knn_dotbrute_"), torch.from_numpy(g["knn_dotbrute_sample"]))
    ours, ref = sample("knn_dot_"), torch.from_numpy(g["knn_dot_sample"])
    assert int((ours != ref).sum()) == 126
    assert (int(ours.sum()), int(ref.sum())) == (100, 122)
