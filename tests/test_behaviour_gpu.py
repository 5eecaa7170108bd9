"""The reference's behavioural hot-path tests, ported onto the HIP product
(graphs drawn from θ by the HIP sampler, aggregations and their θ-gradients
on the HIP kernels) on the real Cora fixture:

  tst/trainers/test_inner_trainer.py:35-41   every parameter changes (lr = 1.0)
  tst/trainers/test_inner_trainer.py:44-53   backprop through time: the graph of
                                             step 1 gets a gradient after 3 steps
  tst/trainers/test_inner_trainer.py:56-70   detach() truncates: graph 1 none,
                                             graph 2 a gradient
  tst/trainers/test_inner_trainer.py:73-81   train accuracy rises for 10 steps
  tst/models/test_bernoulli_model.py:101-110 the gradient through sample()
                                             reaches every θ entry (the
                                             straight-through estimator's dense
                                             gradient; only the diagonal, whose
                                             self-loop is SET, gets none)
  tst/models/test_gcn.py:75-109              params= overrides the forward and
                                             its gradients go only to the
                                             override dict

The reference marks graphs by requires_grad on dense matrices; here a graph's
gradient lands on the θ it was drawn from, so each graph gets its own
BernoulliGraphModel and "graph k has a gradient" reads θ_k.grad."""
import pytest
import torch

import ldsgnn
from ldsgnn.models.gcn import MetaDenseGCN
from ldsgnn.models.graph import BernoulliGraphModel
from ldsgnn.trainers.inner import InnerProblemTrainer

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def cora():
    """The reference tests' fixture: Planetoid Cora + CreateDenseAdjacencyMatrix,
    raw features (tst/trainers/test_inner_trainer.py:19-22, no NormalizeFeatures)."""
    from ldsgnn.data.planetoid import load_planetoid_npz
    return load_planetoid_npz("cora", normalize_features=False).to(DEV)


def _model(data, dropout=0.0):
    torch.manual_seed(42)
    ldsgnn.rng.manual_seed(42, 0)
    return MetaDenseGCN(data.num_features, 16, data.num_classes, dropout=dropout).to(DEV)


def _graph_model(data, scale=1.0):
    return _theta_model(data.dense_adj, scale)


def _theta_model(adj, scale):
    gm = BernoulliGraphModel(adj)
    with torch.no_grad():
        gm.probs.mul_(scale).add_((1.0 - scale) * 0.5)  # fractional θ: every entry can be drawn either way
    return gm


def test_all_parameters_change(cora):
    trainer = InnerProblemTrainer(_model(cora), data=cora, lr=1.0)
    init = [p.detach().clone() for p in trainer.model_params.values()]
    trainer.train_step(_graph_model(cora).sample())
    for a, b in zip(init, trainer.model_params.values()):
        assert (a != b.detach()).all()


def test_backprop_through_time_works(cora):
    trainer = InnerProblemTrainer(_model(cora), data=cora, lr=1.0)
    g1 = _graph_model(cora, 0.9)
    other = _graph_model(cora, 0.5)
    trainer.train_step(g1.sample())
    trainer.train_step(other.sample())
    trainer.train_step(other.sample())
    trainer.model_forward(other.sample()).sum().backward()
    assert g1.probs.grad is not None and bool((g1.probs.grad != 0).any())


def test_detach_works(cora):
    trainer = InnerProblemTrainer(_model(cora), data=cora, lr=1.0)
    g1, g2 = _graph_model(cora, 0.9), _graph_model(cora, 0.8)
    other = _graph_model(cora, 0.5)
    trainer.train_step(g1.sample())
    trainer.train_step(other.sample())
    trainer.detach()
    trainer.train_step(g2.sample())
    trainer.train_step(other.sample())
    trainer.model_forward(other.sample()).sum().backward()
    assert g1.probs.grad is None
    assert g2.probs.grad is not None and bool((g2.probs.grad != 0).any())


def test_model_acc_improves(cora):
    trainer = InnerProblemTrainer(_model(cora), data=cora, lr=0.001)
    graph = cora.dense_adj.clone()  # the fixed graph: hot-path CSR via MetaDenseGCN.fixed_graph
    acc = 0.0
    for _ in range(10):
        m = trainer.train_step(graph)
        assert m.acc > acc
        acc = m.acc


def test_gradient_through_sample_reaches_every_theta_entry(cora):
    n = 300
    a = cora.dense_adj[:n, :n].contiguous()
    gm = _theta_model(a, 0.8)
    assert gm.probs.grad is None
    graph = gm.sample()
    torch.manual_seed(0)
    gcn = MetaDenseGCN(12, 16, 5, dropout=0.0).to(DEV)
    x = torch.rand(n, 12, device=DEV)
    w = torch.randn(n, 5, device=DEV)
    (gcn(x, graph) * w).sum().backward()
    g = gm.probs.grad
    assert g is not None
    idx = torch.arange(n, device=DEV)
    diag = idx * (2 * n - idx + 1) // 2
    off = torch.ones_like(g, dtype=torch.bool)
    off[diag] = False
    assert bool((g[off] != 0).all())      # dense straight-through gradient, every off-diagonal entry
    assert bool((g[diag] == 0).all())     # self-loops are set, not drawn (tst/utils/test_graph.py:169-178)


def test_meta_dense_gcn_overrides_params(cora):
    gcn = _model(cora, dropout=0.5)
    graph = _graph_model(cora, 0.9).sample()
    gcn.eval()
    zero = {k: torch.zeros_like(p) for k, p in gcn.named_parameters()}
    assert not torch.equal(gcn(cora.x, graph), gcn(cora.x, graph, params=zero))


def test_meta_dense_gcn_overridden_params_trainable(cora):
    gcn = _model(cora, dropout=0.5)
    gm = _graph_model(cora, 0.9)
    over = {k: torch.rand_like(p).requires_grad_(True) for k, p in gcn.named_parameters()}
    gcn(cora.x, gm.sample(), params=over).sum().backward()
    for p in gcn.parameters():
        assert p.grad is None
    for p in over.values():
        assert p.grad is not None
    assert gm.probs.grad is not None
