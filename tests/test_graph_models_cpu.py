"""Host-side pieces of the embedding / GAE graph models
that need no GPU: the kNN pattern with the reference's metrics, the dense
sparsification semantics, the factory's error behaviour."""
import pytest
import torch

from ldsgnn.models.factory import GraphGenerativeModelFactory
from ldsgnn.models.sampling import SPARSIFICATION, sparsify
from ldsgnn.utils.graph import DenseData, knn_graph_dense


def test_knn_dot_metric_is_a_distance():
    """np.dot passed to sklearn as a metric is read as a distance: the k
    smallest dot products are the neighbours (src/models/sampling.py:30-32)."""
    x = torch.tensor([[1.0, 0.0], [2.0, 0.0], [-1.0, 0.0], [0.0, 1.0]])
    a = knn_graph_dense(x, 1, loop=False, metric="dot")
    # row 0: dots with rows 1..3 = 2, -1, 0 -> nearest is row 2
    assert torch.equal(a[0], torch.tensor([0.0, 0.0, 1.0, 0.0]))
    c = knn_graph_dense(x, 1, loop=False, metric="cosine")
    assert torch.equal(c[0], torch.tensor([0.0, 1.0, 0.0, 0.0]))


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
