"""Generate the golden vectors in tests/golden/*.npz from the REFERENCE CODE.

Run in the development container only (needs /root/reference; the GPU box
never sees the reference):  python tests/golden/make_golden.py

How the reference is run here
  * /root/reference/src is imported as-is.  Its third-party imports that are
    not installed are satisfied by stubs written to a temporary directory
    outside the repository:
      - import-only placeholders (never called on this path): sacred,
        torch_geometric, torch_scatter;
      - functional stand-ins for the two libraries whose arithmetic IS on the
        path, loaded from this repository's restatements:
          torchmeta.modules{,.utils}  <- lds-gnn_amd/ldsgnn/models/meta.py
          higher.optim                <- lds-gnn_amd/ldsgnn/optim.py
        (higher's first-order values are additionally pinned against
        torch.optim.Adam, golden `adam_first_order`).
  * Randomness: `Bernoulli` in src.models.sampling and `F.dropout` in
    src.models.gcn are replaced by draws from the keyed Philox map
    (oracle/philox.py) on the product's schedule (ldsgnn/rng.py), so the GPU
    product and the reference see identical edge sets and dropout masks.  One
    golden (`sampling_native`) keeps torch's own RNG to pin the injected-U mode.
Nothing from the reference is copied into the repository: only inputs and
outputs (arrays) are stored.
"""
from __future__ import annotations

import importlib.util
import os
import sys
import tempfile
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, ROOT)
from oracle import philox  # noqa: E402

TAG_GRAPH, TAG_DROP_X, TAG_DROP_H = philox.TAG_GRAPH, philox.TAG_DROP_X, philox.TAG_DROP_H


# ---------------------------------------------------------------------------
# stubs
# ---------------------------------------------------------------------------

def _load_file_module(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def install_stubs():
    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    class Ingredient:
        def __init__(self, *a, **k):
            pass

        def config(self, f):
            return f

        def capture(self, f):
            return f

    class _Placeholder:
        def __init__(self, *a, **k):
            raise RuntimeError("stub placeholder called: not on the golden path")

    class Data:
        def __init__(self, **kwargs):
            for k, v in kwargs.items():
                setattr(self, k, v)

    mod("sacred", Ingredient=Ingredient, Experiment=_Placeholder)
    mod("sacred.observers", TelegramObserver=_Placeholder)
    mod("sacred.run", Run=object)
    mod("torch_geometric")
    mod("torch_geometric.data", Data=Data)
    mod("torch_geometric.datasets", Planetoid=_Placeholder)
    mod("torch_geometric.nn")
    mod("torch_geometric.nn.models", GAE=_Placeholder)
    mod("torch_geometric.transforms", NormalizeFeatures=_Placeholder, Compose=_Placeholder)
    mod("torch_geometric.utils", to_scipy_sparse_matrix=_Placeholder, to_undirected=_Placeholder)
    mod("torch_scatter", scatter_add=_Placeholder)
    meta = _load_file_module("ldsgnn_meta_standin", os.path.join(ROOT, "lds-gnn_amd/ldsgnn/models/meta.py"))
    mod("torchmeta")
    mod("torchmeta.modules", MetaModule=meta.MetaModule, MetaLinear=meta.MetaLinear)
    mod("torchmeta.modules.utils", get_subdict=meta.get_subdict)
    opt = _load_file_module("ldsgnn_optim_standin", os.path.join(ROOT, "lds-gnn_amd/ldsgnn/optim.py"))
    mod("higher")
    mod("higher.optim", DifferentiableOptimizer=opt.DifferentiableOptimizer,
        DifferentiableAdam=opt.DifferentiableAdam)
    if REF not in sys.path:
        sys.path.insert(0, REF)


# ---------------------------------------------------------------------------
# keyed randomness patched into the reference
# ---------------------------------------------------------------------------

class KeyedRandomness:
    """The product's draw schedule (ldsgnn/rng.py) as patches on the reference."""

    def __init__(self, seed: int, replica: int = 0):
        self.seed, self.replica = seed, replica
        self.graph_counter = 0
        self.forward_counter = 0
        self._pending_h = None

    def bernoulli_class(self):
        outer = self

        class Bernoulli:
            def __init__(self, probs):
                self.probs = probs

            def sample(self):
                n = self.probs.size(0)
                c = outer.graph_counter
                outer.graph_counter += 1
                u = philox.uniform(outer.seed, philox.tag_for(TAG_GRAPH, outer.replica), c, n, n)
                return (torch.from_numpy(u) < self.probs.detach()).to(self.probs.dtype)

        return Bernoulli

    def functional(self):
        import torch.nn.functional as F
        outer = self

        def dropout(x, p=0.5, training=True, inplace=False):
            if not training or p == 0.0:
                return x
            if outer._pending_h is None:
                c = outer.forward_counter
                outer.forward_counter += 1
                tag = philox.tag_for(TAG_DROP_X, outer.replica)
                outer._pending_h = c
            else:
                c = outer._pending_h
                tag = philox.tag_for(TAG_DROP_H, outer.replica)
                outer._pending_h = None
            u = torch.from_numpy(philox.uniform(outer.seed, tag, c, x.size(0), x.size(1)))
            keep = np.float32(1.0) - np.float32(p)
            return x * ((u < float(keep)).to(x.dtype) * float(np.float32(1.0) / keep))

        proxy = types.SimpleNamespace(**{k: getattr(F, k) for k in dir(F) if not k.startswith("__")})
        proxy.dropout = dropout
        return proxy


def patch_reference(rnd: KeyedRandomness):
    import src.models.gcn as gcn_mod
    import src.models.sampling as sampling_mod
    sampling_mod.Bernoulli = rnd.bernoulli_class()
    gcn_mod.F = rnd.functional()
    # sacred would inject the sampler config (src/models/sampling.py:96-102)
    sampling_mod.Sampler.sample = staticmethod(_sampler_with_config(sampling_mod))


def _sampler_with_config(sampling_mod):
    def sample(edge_probs, undirected=True, sparsification="NONE", k=20, eps=0.9, embeddings=None,
               dense=False, knn_metric="cosine"):
        return sampling_mod.sample_graph(edge_probs=edge_probs, embeddings=embeddings, undirected=undirected,
                                         sparsification=sampling_mod.SPARSIFICATION[sparsification],
                                         dense=dense, k=k, eps=eps, knn_metric=knn_metric)
    return sample


# ---------------------------------------------------------------------------
# problems
# ---------------------------------------------------------------------------

def synthetic(n, f_in, classes, seed, p_edge=0.05):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(n, f_in, generator=g) * (torch.rand(n, f_in, generator=g) < 0.3)
    x = x / x.sum(1, keepdim=True).clamp(min=1e-12)
    y = torch.randint(0, classes, (n,), generator=g)
    perm = torch.randperm(n, generator=g)
    ntr, nva = max(2, n // 5), max(2, (3 * n) // 10)
    masks = []
    for idx in (perm[:ntr], perm[ntr:ntr + nva // 2], perm[ntr + nva // 2:ntr + nva], perm[ntr + nva:]):
        m = torch.zeros(n, dtype=torch.bool)
        m[idx] = True
        masks.append(m)
    a = (torch.rand(n, n, generator=g) < p_edge).float().triu(1)
    return dict(x=x, y=y, train=masks[0], val=masks[1], opt=masks[2], test=masks[3], adj=a + a.t())


def dense_data(prob):
    from src.utils.graph import DenseData
    d = DenseData.__new__(DenseData)
    d.x, d.y, d.dense_adj = prob["x"], prob["y"], prob["adj"]
    d.train_mask, d.val_mask, d.test_mask = prob["train"], prob["val"], prob["test"]
    d.num_classes = int(prob["y"].max()) + 1
    return d


def np_prob(prob, prefix=""):
    return {prefix + k: (v.numpy() if isinstance(v, torch.Tensor) else v) for k, v in prob.items()}


def build_reference(prob, seed, dropout, hidden=16, gcn_lr=0.01, gcn_wd=5e-4, outer_lr=0.1, lr_decay=0.99):
    from src.models.gcn import MetaDenseGCN
    from src.models.graph import BernoulliGraphModel
    from src.trainers.bilevel import BilevelProblemRunner
    from src.trainers.inner import InnerProblemTrainer
    from src.trainers.outer import OuterProblemTrainer
    data = dense_data(prob)
    torch.manual_seed(seed)
    gcn = MetaDenseGCN(data.x.size(1), hidden, data.num_classes, dropout=dropout)
    inner = InnerProblemTrainer(gcn, data, lr=gcn_lr, weight_decay=gcn_wd)
    gm = BernoulliGraphModel(data.dense_adj)
    opt = torch.optim.SGD(gm.parameters(), lr=outer_lr)
    outer = OuterProblemTrainer(opt, data, prob["opt"], gm, smoothness_factor=0.0, disconnection_factor=0.0,
                                sparsity_factor=0.0, regularize=False, lr_decay=lr_decay, pretrain=False)
    runner = BilevelProblemRunner(inner, outer, data, n_samples_empirical_mean=16)
    runner.logger = types.SimpleNamespace(info=lambda *a, **k: None, warn=lambda *a, **k: None)
    return runner


class Log:
    def __init__(self):
        self.rows = []

    def log_scalar(self, name, value, step=None):
        self.rows.append((name, float(value), -1 if step is None else int(step)))


# ---------------------------------------------------------------------------
# goldens
# ---------------------------------------------------------------------------

def g_graph_math(out):
    from src.models.sampling import sample_graph, SPARSIFICATION
    from src.utils.graph import normalize_adjacency_matrix, triu_values_to_symmetric_matrix
    g = torch.Generator().manual_seed(1)
    theta8 = torch.rand(36, generator=g) * 1.4 - 0.2
    out["theta8"] = theta8.numpy()
    out["p8"] = triu_values_to_symmetric_matrix(theta8).numpy()
    a = (torch.rand(16, 16, generator=g) < 0.3).float().triu(1)
    a = a + a.t()
    out["adj16"] = a.numpy()
    out["norm16"] = normalize_adjacency_matrix(a).numpy()
    # θ-gradient through P -> sample (STE) -> normalise, reference autograd
    n = 30
    theta = torch.rand(n * (n + 1) // 2, generator=g).requires_grad_(True)
    w = torch.randn(n, n, generator=g)
    p = triu_values_to_symmetric_matrix(theta)
    rnd = KeyedRandomness(seed=4242)
    import src.models.sampling as sm
    old = sm.Bernoulli
    sm.Bernoulli = rnd.bernoulli_class()
    try:
        a30 = sample_graph(p, undirected=True, sparsification=SPARSIFICATION.NONE, dense=False)
    finally:
        sm.Bernoulli = old
    loss = (w * normalize_adjacency_matrix(a30)).sum()
    loss.backward()
    out["theta30"] = theta.detach().numpy()
    out["w30"] = w.numpy()
    out["sample30"] = a30.detach().numpy()
    out["grad30"] = theta.grad.numpy()
    out["seed30"] = np.int64(4242)


def g_sampling_native(out):
    """torch's own RNG: Bernoulli(P).sample() under torch.manual_seed."""
    from src.models.sampling import sample_graph, SPARSIFICATION
    from src.utils.graph import triu_values_to_symmetric_matrix
    import src.models.sampling as sm
    from torch.distributions import Bernoulli as TorchBernoulli
    old = sm.Bernoulli
    sm.Bernoulli = TorchBernoulli
    try:
        n = 64
        g = torch.Generator().manual_seed(2)
        theta = torch.rand(n * (n + 1) // 2, generator=g)
        p = triu_values_to_symmetric_matrix(theta)
        torch.manual_seed(77)
        a = sample_graph(p, undirected=True, sparsification=SPARSIFICATION.NONE, dense=False)
        torch.manual_seed(77)
        u = torch.rand(n, n)
    finally:
        sm.Bernoulli = old
    out["theta"] = theta.numpy()
    out["u"] = u.numpy()
    out["sample"] = a.detach().numpy()


def g_gcn_forward(out):
    from src.models.gcn import MetaDenseGCN
    from src.models.graph import BernoulliGraphModel
    prob = synthetic(64, 20, 5, seed=3, p_edge=0.2)
    rnd = KeyedRandomness(seed=31)
    patch_reference(rnd)
    torch.manual_seed(5)
    gcn = MetaDenseGCN(20, 16, 5, dropout=0.5)
    gm = BernoulliGraphModel(prob["adj"])
    with torch.no_grad():
        gm.probs.mul_(0.5).add_(0.25)  # fractional θ
    graph = gm.sample()
    gcn.train()
    train_out = gcn(prob["x"], graph)
    gcn.eval()
    eval_out = gcn(prob["x"], graph)
    out.update(np_prob(prob, "prob_"))
    out["theta"] = gm.probs.detach().numpy()
    out["params"] = np.concatenate([p.detach().numpy().ravel() for p in gcn.parameters()])
    out["train_logp"] = train_out.detach().numpy()
    out["eval_logp"] = eval_out.detach().numpy()
    out["seed"] = np.int64(31)
    out["torch_seed"] = np.int64(5)


def g_adam_first_order(out):
    """torch.optim.Adam (real torch arithmetic) with the reference's groups on
    the reference GCN: pins the differentiable-Adam restatement's values."""
    from src.models.gcn import MetaDenseGCN
    from src.utils.graph import DenseData  # noqa: F401
    import torch.nn.functional as F
    prob = synthetic(48, 16, 4, seed=4, p_edge=0.1)
    torch.manual_seed(6)
    gcn = MetaDenseGCN(16, 16, 4, dropout=0.0)
    opt = torch.optim.Adam([{"params": gcn.layer_in.parameters(), "weight_decay": 5e-4},
                            {"params": gcn.layer_out.parameters()}], lr=0.01)
    out["params0"] = np.concatenate([p.detach().numpy().ravel() for p in gcn.parameters()])
    traj = []
    for _ in range(5):
        opt.zero_grad()
        pred = gcn(prob["x"], prob["adj"])
        F.nll_loss(pred[prob["train"]], prob["y"][prob["train"]]).backward()
        opt.step()
        traj.append(np.concatenate([p.detach().numpy().ravel() for p in gcn.parameters()]))
    out.update(np_prob(prob, "prob_"))
    out["trajectory"] = np.stack(traj)
    out["torch_seed"] = np.int64(6)


def g_bilevel(out, n=80, f_in=24, classes=4, seed=11, dropout=0.5):
    """The reference's own BilevelProblemRunner.train + evaluate, early
    stopping included, with keyed randomness; θ-gradients of every hyper step."""
    prob = synthetic(n, f_in, classes, seed=seed, p_edge=0.06)
    rnd = KeyedRandomness(seed=seed)
    patch_reference(rnd)
    runner = build_reference(prob, seed=seed, dropout=dropout)
    grads = []
    orig = runner.outer_trainer.train_step

    def spy(*a, **k):
        m = orig(*a, **k)
        grads.append(runner.outer_trainer.model.probs.grad.detach().clone().numpy())
        return m

    runner.outer_trainer.train_step = spy
    log = Log()
    runner.train(patience=3, hyper_gradient_interval=5, inner_loop_max_epochs=12, outer_loop_max_epochs=2,
                 sacred_runner=log)
    res = runner.evaluate()
    out.update(np_prob(prob, "prob_"))
    out["seed"] = np.int64(seed)
    out["dropout"] = np.float64(dropout)
    out["log_names"] = np.array([r[0] for r in log.rows])
    out["log_values"] = np.array([r[1] for r in log.rows])
    out["log_steps"] = np.array([r[2] for r in log.rows])
    out["theta_final"] = runner.outer_trainer.model.probs.detach().numpy()
    out["theta_grads"] = np.stack(grads)
    out["final"] = np.array([res["loss.val.final"], res["acc.val.final"], res["loss.test.final"],
                             res["acc.test.final"]])
    out["graph_draws"] = np.int64(rnd.graph_counter)
    out["forward_draws"] = np.int64(rnd.forward_counter)


def g_conditioning_probe(out):
    """bilevel_small again, with the reference's aggregation torch.mm
    (src/models/layers.py:44) accumulated in fp64 and rounded once — a pure
    rounding change.  Shows how much the reference's own hypergradients move
    under reordered fp32 arithmetic (used to justify whole-loop tolerances)."""
    import src.models.layers as layers
    orig_mm = torch.mm

    class TorchProxy:
        def __getattr__(self, k):
            return getattr(torch, k)

        @staticmethod
        def mm(a, b):
            return orig_mm(a.double(), b.double()).float()

    layers.torch = TorchProxy()
    try:
        g_bilevel(out)
    finally:
        layers.torch = torch


def g_hypergrad_cora(out, seed=7):
    """One τ=5 window on a Cora-shaped problem (N=2708, F_in=1433, C=7):
    5 inner steps + the hyper step, reference code; θ-gradient summary."""
    sys.path.insert(0, os.path.join(ROOT, "lds-gnn_amd"))
    from ldsgnn.data.synthetic import knn_init, make_dataset
    data = knn_init(make_dataset("cora", seed=seed), k=10)
    gperm = torch.Generator().manual_seed(seed)
    val_idx = data.val_mask.nonzero().squeeze(1)
    val_idx = val_idx[torch.randperm(val_idx.numel(), generator=gperm)]
    opt_mask = torch.zeros_like(data.val_mask)
    opt_mask[val_idx[: val_idx.numel() // 2]] = True
    prob = dict(x=data.x, y=data.y, train=data.train_mask, val=data.val_mask & ~opt_mask, opt=opt_mask,
                test=data.test_mask, adj=data.dense_adj)
    rnd = KeyedRandomness(seed=seed)
    patch_reference(rnd)
    runner = build_reference(prob, seed=seed, dropout=0.5)
    losses = []
    for step in range(6):
        losses.append(runner.inner_opt_step().loss)
        if step % 5 == 0:
            runner.hyper_opt_step(step)
    grad = runner.outer_trainer.model.probs.grad.detach().numpy().astype(np.float64)
    theta = runner.outer_trainer.model.probs.detach().numpy()
    pick = np.random.default_rng(seed).choice(grad.size, 20000, replace=False)
    out["seed"] = np.int64(seed)
    out["opt_mask"] = opt_mask.numpy()
    # the data itself travels (kNN near-ties and row sums are machine-dependent)
    xs = data.x.to_sparse_csr()
    out["x_indptr"] = xs.crow_indices().numpy().astype(np.int64)
    out["x_indices"] = xs.col_indices().numpy().astype(np.int32)
    out["x_values"] = xs.values().numpy()
    out["x_shape"] = np.array(data.x.shape)
    iu = torch.triu_indices(data.x.shape[0], data.x.shape[0], 1)
    keep = data.dense_adj[iu[0], iu[1]] != 0
    out["adj_edges"] = iu[:, keep].numpy().astype(np.int32)
    out["y"] = data.y.numpy()
    out["train_mask"] = data.train_mask.numpy()
    out["val_mask"] = data.val_mask.numpy()
    out["test_mask"] = data.test_mask.numpy()
    out["inner_losses"] = np.array(losses)
    out["grad_idx"] = pick.astype(np.int64)
    out["grad_val"] = grad[pick].astype(np.float32)
    out["grad_sum"] = grad.sum()
    out["grad_l2"] = np.sqrt((grad ** 2).sum())
    out["theta_idx"] = pick.astype(np.int64)
    out["theta_val"] = theta[pick]
    out["theta_sum"] = theta.astype(np.float64).sum()


def _planetoid(name):
    """The real Planetoid split from the committed fixture, NormalizeFeatures
    and MakeUndirected applied (ldsgnn.data.planetoid, pinned by
    tests/test_planetoid.py against the reference's own data facts)."""
    sys.path.insert(0, os.path.join(ROOT, "lds-gnn_amd"))
    from ldsgnn.data.planetoid import load_planetoid_npz
    return load_planetoid_npz(name)


def _triu_edges(adj):
    n = adj.size(0)
    iu = torch.triu_indices(n, n, 1)
    keep = adj[iu[0], iu[1]] != 0
    return iu[:, keep].numpy().astype(np.int32)


def _adj_from_edges(n, edges):
    a = torch.zeros(n, n)
    e = torch.from_numpy(edges).long()
    a[e[0], e[1]] = 1.0
    a[e[1], e[0]] = 1.0
    return a


def g_knn_cora(out):
    """θ₀ of BASELINE config 2: the reference's own knn_graph_dense
    (src/data/utils.py:165-175, sklearn kneighbors_graph, k=10, cosine,
    include_self=False as KNNGraph(loop=False) passes it,
    src/data/dataloader.py:104-105) on the real Cora features after
    NormalizeFeatures, then MakeUndirected (src/data/transforms.py:31-37)."""
    import sklearn
    from src.data.utils import knn_graph_dense as reference_knn
    data = _planetoid("cora")
    a = reference_knn(data.x, 10, loop=False, metric="cosine")
    out["directed"] = np.stack(np.nonzero(a.numpy())).astype(np.int32)  # row i -> its 10 nearest
    out["edges"] = _triu_edges(torch.max(a, a.t()))                       # undirected, i < j
    out["k"] = np.int64(10)
    out["sklearn_version"] = np.array(sklearn.__version__)


def _spy_grads(runner, grads):
    orig = runner.outer_trainer.train_step

    def spy(*a, **k):
        m = orig(*a, **k)
        grads.append(runner.outer_trainer.model.probs.grad.detach().clone().numpy().astype(np.float64))
        return m

    runner.outer_trainer.train_step = spy


def _store_vec(out, key, v, pick):
    out[key + "_val"] = v[pick].astype(np.float32)
    out[key + "_sum"] = np.float64(v.astype(np.float64).sum())
    out[key + "_l2"] = np.float64(np.sqrt((v.astype(np.float64) ** 2).sum()))


def _opt_split(data, seed):
    """bilevel.py:77: split_mask(val_mask, 0.5, shuffle=True) with numpy's
    global RNG seeded (the reference's own split_mask)."""
    from src.utils.graph import split_mask
    np.random.seed(seed)
    return split_mask(data.val_mask, 0.5, shuffle=True)


def g_hypergrad_cora_real(out, seed=11):
    """BASELINE config 2 exactly: real Cora, kNN θ₀ (golden knn_cora), the
    reference's first two hyper steps (step 0: a 1-step window; steps 1-5: the
    τ=5 window) with dropout 0.5, SGD lr 0.1, decay 0.99."""
    data = _planetoid("cora")
    knn = np.load(os.path.join(HERE, "knn_cora.npz"))
    adj = _adj_from_edges(data.num_nodes, knn["edges"])
    val, opt = _opt_split(data, seed)
    prob = dict(x=data.x, y=data.y, train=data.train_mask, val=val, opt=opt, test=data.test_mask, adj=adj)
    rnd = KeyedRandomness(seed=seed)
    patch_reference(rnd)
    runner = build_reference(prob, seed=seed, dropout=0.5)
    grads, losses, thetas = [], [], []
    _spy_grads(runner, grads)
    for step in range(6):
        losses.append(runner.inner_opt_step().loss)
        if step % 5 == 0:
            runner.hyper_opt_step(step)
            thetas.append(runner.outer_trainer.model.probs.detach().clone().numpy())
    pick = np.random.default_rng(seed).choice(grads[0].size, 20000, replace=False)
    out["seed"] = np.int64(seed)
    out["opt_mask"] = opt.numpy()
    out["val_mask"] = val.numpy()
    out["inner_losses"] = np.array(losses)
    out["idx"] = pick.astype(np.int64)
    for h in range(2):
        _store_vec(out, f"grad{h}", grads[h], pick)
        _store_vec(out, f"theta{h}", thetas[h], pick)
    params = runner.inner_trainer.model_params
    out["params_final"] = np.concatenate([params[k].detach().numpy().ravel() for k in params])


def g_hypergrad_cora_wellcond(out, seed=11):
    """Two well-conditioned θ-gradients at BASELINE config 2's size (real
    Cora, kNN θ₀), where no Adam step sits between θ and the loss, so rounding
    is not amplified (unlike hypergrad_cora_real's windows):
      outer: the reference's step-0 window (dropout 0.5), then a hyper step
             with NO inner step before it — NLL on the opt mask through one
             sampled outer graph with the weights as leaves
             (src/trainers/outer.py:57-87 after bilevel.py:109-114's detach);
      nd:    the same real-Cora run with dropout 0 (every forward
             deterministic given its graph): the step-0 window, its
             outer-only hyper step, then a dropout-free τ = 5 window.
    Stored per gradient: 20 000 picked entries, sum and L2 norm."""
    data = _planetoid("cora")
    knn = np.load(os.path.join(HERE, "knn_cora.npz"))
    adj = _adj_from_edges(data.num_nodes, knn["edges"])
    val, opt = _opt_split(data, seed)
    prob = dict(x=data.x, y=data.y, train=data.train_mask, val=val, opt=opt, test=data.test_mask, adj=adj)
    out["seed"] = np.int64(seed)
    out["opt_mask"] = opt.numpy()
    out["val_mask"] = val.numpy()
    for tag, dropout in (("", 0.5), ("nd_", 0.0)):
        rnd = KeyedRandomness(seed=seed)
        patch_reference(rnd)
        runner = build_reference(prob, seed=seed, dropout=dropout)
        grads, thetas = [], []
        _spy_grads(runner, grads)
        loss0 = runner.inner_opt_step().loss
        runner.hyper_opt_step(0)
        thetas.append(runner.outer_trainer.model.probs.detach().clone().numpy())
        runner.hyper_opt_step(1)  # no inner step in this window: the outer graph's path only
        thetas.append(runner.outer_trainer.model.probs.detach().clone().numpy())
        keys = ["grad_step0", "grad_outer"]
        if dropout == 0.0:  # then a whole τ = 5 window (steps 1-5)
            losses = [runner.inner_opt_step().loss for _ in range(5)]
            runner.hyper_opt_step(5)
            thetas.append(runner.outer_trainer.model.probs.detach().clone().numpy())
            keys.append("grad_window")
            out[tag + "window_losses"] = np.array(losses)
        if "idx" not in out:
            out["idx"] = np.random.default_rng(seed).choice(grads[0].size, 20000, replace=False).astype(np.int64)
        pick = out["idx"]
        out[tag + "inner_loss0"] = np.float64(loss0)
        for h, key in enumerate(keys):
            _store_vec(out, tag + key, grads[h], pick)
            _store_vec(out, tag + key.replace("grad", "theta"), thetas[h], pick)
        params = runner.inner_trainer.model_params
        out[tag + "params"] = np.concatenate([params[k].detach().numpy().ravel() for k in params])


def g_graph_models(out):
    """SURVEY §8(f) item 4 by the reference code itself (src/models/graph.py:
    81-200, src/models/sampling.py:19-85), on the keyed Philox uniforms
    (stored as `u_*`, injected into the product's sampler):
      emb_*   PairwiseEmbeddingSampler (n 70, d 8, prob_pow 1 and 2):
              forward() P, sample() (the sacred default: undirected, NONE,
              STE) and dE of L = Σ (normalize(A_ste)·Z) ⊙ W;
      knn_*   sample_graph with KNN sparsification (k 7) on the embeddings,
              cosine and np.dot (the reference passes np.dot to sklearn as a
              callable metric, i.e. as a distance), and dE through it; for
              np.dot also with sklearn's exact brute-force search (knn_dotbrute:
              the default BallTree is not exact on a non-metric);
      eps_*   sample_graph with EPS (eps 0.5, 1.5) on the draw, and the
              dense=True EPS rule on the probabilities;
      gae_*   GraphProposalNetwork.calculate_edges_and_embeddings (n 48,
              f_in 12, embedding 8, dropout 0; normalised similarities /
              add_original) with its GCN weights, P and embeddings, and the
              gradients of L through one STE sample to the GCN weights,
              probs_factor and probs_bias (plus the fp64 rerun of the same
              gradient: the reference's own conditioning probe)."""
    import src.models.sampling as sm
    from src.models.graph import GraphProposalNetwork, PairwiseEmbeddingSampler
    from src.utils.graph import normalize_adjacency_matrix
    rnd = KeyedRandomness(seed=61)
    patch_reference(rnd)

    def uniforms(n):  # the next Bernoulli draw's uniforms (graph counter rnd.graph_counter)
        return philox.uniform(rnd.seed, philox.tag_for(TAG_GRAPH, rnd.replica), rnd.graph_counter, n, n)

    def loss_of(a, z, w):
        return ((normalize_adjacency_matrix(a) @ z) * w).sum()

    g = torch.Generator().manual_seed(3)
    n, d = 70, 8
    e0 = torch.rand(n, d, generator=g) * 2 - 1
    z = torch.randn(n, 16, generator=g)
    w = torch.randn(n, 16, generator=g)
    out["emb_e"], out["emb_z"], out["emb_w"] = e0.numpy(), z.numpy(), w.numpy()
    for pw in (1.0, 2.0):
        key = f"emb_pow{int(pw)}_"
        m = PairwiseEmbeddingSampler(n_nodes=n, embedding_dim=d, prob_pow=pw)
        with torch.no_grad():
            m.embeddings.copy_(e0)
        out[key + "p"] = m.forward().detach().numpy()
        out[key + "u"] = uniforms(n)
        a = m.sample()
        out[key + "sample"] = a.detach().numpy()
        loss_of(a, z, w).backward()
        out[key + "grad_e"] = m.embeddings.grad.detach().numpy()
    ref_knn = sm.knn_graph_dense

    def knn_brute(x, k, loop=True, metric="cosine"):
        # the reference's knn_graph_dense (src/data/utils.py:165-175) with
        # sklearn's exact brute-force search: with metric=np.dot sklearn's
        # default picks a BallTree, whose pruning is not exact on a
        # non-metric (negative "distances")
        from sklearn.neighbors import NearestNeighbors
        nn = NearestNeighbors(n_neighbors=k, metric=metric, algorithm="brute").fit(x.numpy())
        return torch.FloatTensor(nn.kneighbors_graph(None if not loop else x.numpy(), n_neighbors=k,
                                                     mode="connectivity").toarray())

    for metric, knn in (("cosine", ref_knn), ("dot", ref_knn), ("dotbrute", knn_brute)):
        key = f"knn_{metric}_"
        sm.knn_graph_dense = knn
        e = e0.clone().requires_grad_(True)
        p = torch.sigmoid(e @ e.t())
        out[key + "u"] = uniforms(n)
        a = sm.sample_graph(p, undirected=True, embeddings=e, dense=False, k=7,
                            sparsification=sm.SPARSIFICATION.KNN, knn_metric=metric[:3] if metric != "cosine"
                            else metric)
        out[key + "sample"] = a.detach().numpy()
        loss_of(a, z, w).backward()
        out[key + "grad_e"] = e.grad.detach().numpy()
    sm.knn_graph_dense = ref_knn
    pe = torch.sigmoid(e0[:50] @ e0[:50].t())
    out["eps_p"] = pe.numpy()
    for eps in (0.5, 1.5):
        key = f"eps_{str(eps).replace('.', 'p')}_"
        out[key + "u"] = uniforms(50)
        a = sm.sample_graph(pe, undirected=True, dense=False, sparsification=sm.SPARSIFICATION.EPS, eps=eps)
        out[key + "sample"] = a.detach().numpy()
    pd = pe.clone().requires_grad_(True)
    a = sm.sample_graph(pd, undirected=True, dense=True, sparsification=sm.SPARSIFICATION.EPS, eps=0.6)
    a.sum().backward()
    out["eps_dense"], out["eps_dense_grad"] = a.detach().numpy(), pd.grad.numpy()

    n, f_in, emb = 48, 12, 8
    g = torch.Generator().manual_seed(21)
    x = torch.rand(n, f_in, generator=g)
    adj = (torch.rand(n, n, generator=g) < 0.1).float()
    adj = torch.maximum(adj, adj.t())
    adj.fill_diagonal_(0.0)
    z = torch.randn(n, 16, generator=g)
    w = torch.randn(n, 16, generator=g)
    out["gae_x"], out["gae_adj"], out["gae_z"], out["gae_w"] = x.numpy(), adj.numpy(), z.numpy(), w.numpy()
    for tag, normalize, add_original in (("cos", True, False), ("dot", False, True)):
        key = f"gae_{tag}_"
        torch.manual_seed(4)
        m = GraphProposalNetwork(x, adj, dropout=0.0, add_original=add_original, embedding_dim=emb,
                                 probs_bias_init=-0.5, probs_factor_init=2.0, normalize_similarities=normalize)
        out[key + "params"] = np.concatenate([q.detach().numpy().ravel() for q in m.gcn.parameters()])
        p, e = m.calculate_edges_and_embeddings()
        out[key + "p"], out[key + "emb"] = p.detach().numpy(), e.detach().numpy()
        out[key + "u"] = uniforms(n)
        a = m.sample()
        out[key + "sample"] = a.detach().numpy()
        loss_of(a, z, w).backward()
        out[key + "grad_params"] = np.concatenate([q.grad.numpy().ravel() for q in m.gcn.parameters()])
        out[key + "grad_factor"] = np.float64(m.probs_factor.grad)
        out[key + "grad_bias"] = np.float64(m.probs_bias.grad)
        # conditioning probe: the same reference computation in fp64 (same
        # weights, same sample).  With normalised similarities near 1 the
        # reference's own fp32 gradient moves by ~1e-4 of its max under it.
        m64 = GraphProposalNetwork(x.double(), adj.double(), dropout=0.0, add_original=add_original,
                                   embedding_dim=emb, probs_bias_init=-0.5, probs_factor_init=2.0,
                                   normalize_similarities=normalize).double()
        with torch.no_grad():
            for q64, q in zip(m64.gcn.parameters(), m.gcn.parameters()):
                q64.copy_(q.double())
        p64, _ = m64.calculate_edges_and_embeddings()
        a64 = (torch.from_numpy(out[key + "sample"]).double() - p64).detach() + p64
        ((normalize_adjacency_matrix(a64) @ z.double()) * w.double()).sum().backward()
        out[key + "grad_params_fp64"] = np.concatenate([q.grad.numpy().ravel() for q in m64.gcn.parameters()])


class _Fp64Products:
    """The reference's two matrix products — the aggregation torch.mm
    (src/models/layers.py:44) and the linear layers' F.linear (torchmeta
    MetaLinear) — accumulated in fp64 and rounded once: a pure rounding
    change, for the conditioning probes."""

    def __enter__(self):
        import src.models.layers as layers
        import torch.nn.functional as F
        orig_mm = torch.mm

        class TorchProxy:
            def __getattr__(self, k):
                return getattr(torch, k)

            @staticmethod
            def mm(a, b):
                return orig_mm(a.double(), b.double()).float()

        f_linear = types.SimpleNamespace(**{k: getattr(F, k) for k in dir(F) if not k.startswith("__")})
        f_linear.linear = lambda x, w, b=None: F.linear(x.double(), w.double(),
                                                        None if b is None else b.double()).float()
        # the globals of torchmeta's MetaLinear stand-in (F.linear)
        self.glob = sys.modules["torchmeta.modules"].MetaLinear.forward.__globals__
        self.layers, self.F = layers, F
        layers.torch, self.glob["F"] = TorchProxy(), f_linear
        return self

    def __exit__(self, *exc):
        self.layers.torch, self.glob["F"] = torch, self.F


def g_hypergrad_cora_real_probe(out):
    """hypergrad_cora_real again under _Fp64Products.  How far the reference's
    OWN hypergradients move under reordered fp32 arithmetic at config 2 bounds
    what any other correct fp32 implementation can be held to: higher's Adam
    update lr·m̂/(√v̂ + eps) has derivative up to lr/eps = 10⁶ in g for
    parameters with |g| near eps (at the first Adam step it is ≈ lr·sign(g)),
    so the hypergradient amplifies the rounding of those gradients
    (DESIGN §6)."""
    with _Fp64Products():
        g_hypergrad_cora_real(out)


def g_hypergrad_citeseer_s16_probe(out):
    """hypergrad_citeseer_s16 again under _Fp64Products (config 3's probe)."""
    with _Fp64Products():
        g_hypergrad_citeseer_s16(out)


def g_hypergrad_citeseer_s16(out, seed=13, samples=16):
    """BASELINE config 3: real Citeseer, θ₀ = the given graph, S = 16
    Monte-Carlo replicas.  Replica b is the reference's own runner with the
    keyed stream of replica b (tags + b) and the same initial GCN (same torch
    seed); each runs one τ=5 window (5 inner steps + its hyper step) from θ₀.
    The engine's batched window moves θ by the MEAN of the 16 hypergradients
    (SURVEY §8(e)), stored here with θ₁ = clamp(θ₀ − 0.1·mean, 0, 1)."""
    data = _planetoid("citeseer")
    val, opt = _opt_split(data, seed)
    prob = dict(x=data.x, y=data.y, train=data.train_mask, val=val, opt=opt, test=data.test_mask,
                adj=data.dense_adj)
    mean, losses, outer = None, [], []
    theta0 = None
    for b in range(samples):
        rnd = KeyedRandomness(seed=seed, replica=b)
        patch_reference(rnd)
        runner = build_reference(prob, seed=seed, dropout=0.5)
        if theta0 is None:
            theta0 = runner.outer_trainer.model.probs.detach().clone()
        grads = []
        _spy_grads(runner, grads)
        losses.append([runner.inner_opt_step().loss for _ in range(5)])
        m = runner.outer_trainer.train_step(runner.inner_trainer.model_forward)
        outer.append(m.loss)
        mean = grads[0] if mean is None else mean + grads[0]
        print(f"  citeseer replica {b}: inner {losses[-1][-1]:.6f} outer {m.loss:.6f}", flush=True)
    mean /= samples
    theta1 = (theta0 - 0.1 * torch.from_numpy(mean).float()).clamp(0.0, 1.0).numpy()
    pick = np.random.default_rng(seed).choice(mean.size, 20000, replace=False)
    out["seed"] = np.int64(seed)
    out["samples"] = np.int64(samples)
    out["opt_mask"] = opt.numpy()
    out["val_mask"] = val.numpy()
    out["inner_losses"] = np.array(losses)   # [S, 5]
    out["outer_losses"] = np.array(outer)    # [S]
    out["idx"] = pick.astype(np.int64)
    _store_vec(out, "grad", mean, pick)
    _store_vec(out, "theta1", theta1, pick)


def g_hypergrad_citeseer_s16_wellcond(out, seed=13, samples=16):
    """BASELINE config 3's shape (real Citeseer, θ₀ = the given graph, S = 16
    replicas, replica b on the keyed stream of replica b) without dropout, in
    the construction of hypergrad_cora_wellcond's dropout-free run:
      step0:  the step-0 window (one inner step, its hyper step);
      outer:  a hyper step with NO inner step before it (NLL on the opt mask
              through each replica's sampled outer graph, the weights as
              leaves): no Adam step between θ and the loss;
      window: a dropout-free τ = 5 window.
    The 16 reference runners are kept side by side, each with its own keyed
    stream (patched in before each of its steps); after every hyper step all
    replicas' θ are set to clamp(θ − lr · mean_b dθ_b, 0, 1) — the shared θ of
    the engine's batched replicas — with lr the SGD rate that step used."""
    data = _planetoid("citeseer")
    val, opt = _opt_split(data, seed)
    prob = dict(x=data.x, y=data.y, train=data.train_mask, val=val, opt=opt, test=data.test_mask,
                adj=data.dense_adj)
    rnds = [KeyedRandomness(seed=seed, replica=b) for b in range(samples)]
    runners, grads = [], [[] for _ in range(samples)]
    for b in range(samples):
        patch_reference(rnds[b])
        runners.append(build_reference(prob, seed=seed, dropout=0.0))
        _spy_grads(runners[b], grads[b])

    def synced_hyper(tag):
        theta_old = runners[0].outer_trainer.model.probs.detach().clone()
        lr = runners[0].outer_trainer.optimizer.param_groups[0]["lr"]
        losses = []
        for b in range(samples):
            patch_reference(rnds[b])
            r = runners[b]  # BilevelProblemRunner.hyper_opt_step (src/trainers/bilevel.py:109-113), its loss kept
            losses.append(r.outer_trainer.train_step(r.inner_trainer.model_forward).loss)
            r.inner_trainer.detach()
            r.outer_trainer.detach()
        mean = sum(gb[-1] for gb in grads) / samples
        theta_new = theta_old.add(torch.from_numpy(mean).float(), alpha=-lr).clamp_(0.0, 1.0)
        for r in runners:
            with torch.no_grad():
                r.outer_trainer.model.probs.data.copy_(theta_new)
        if "idx" not in out:
            out["idx"] = np.random.default_rng(seed).choice(mean.size, 20000, replace=False).astype(np.int64)
        _store_vec(out, "grad_" + tag, mean, out["idx"])
        _store_vec(out, "theta_" + tag, theta_new.numpy(), out["idx"])
        out[tag + "_outer_losses"] = np.array(losses)

    def inner_steps(k, tag):
        rows = []
        for b in range(samples):
            patch_reference(rnds[b])
            rows.append([runners[b].inner_opt_step().loss for _ in range(k)])
        out[tag + "_inner_losses"] = np.array(rows)  # [S, k]

    inner_steps(1, "step0")
    synced_hyper("step0")
    synced_hyper("outer")      # no inner step in this window
    inner_steps(5, "window")
    synced_hyper("window")
    print("  citeseer nd window outer losses", out["window_outer_losses"][:4], flush=True)
    out["seed"] = np.int64(seed)
    out["samples"] = np.int64(samples)
    out["opt_mask"] = opt.numpy()
    out["val_mask"] = val.numpy()


def g_gcn_fixed_cora(out, seed=17, epochs=200, patience=10):
    """BASELINE config 1: the reference's fixed-graph GCN training loop
    (src/scripts/gcn.py:56-99 statement for statement: Adam groups 62-67,
    train / backward / step / evaluate / EarlyStopping on val.loss) on the
    real Cora split and given graph, dropout 0.5 from the keyed stream."""
    from src.models.gcn import MetaDenseGCN
    from src.utils.early_stopping import EarlyStopping
    from src.utils.evaluation import accuracy, evaluate
    import torch.nn.functional as F
    data = _planetoid("cora")
    rnd = KeyedRandomness(seed=seed)
    patch_reference(rnd)
    torch.manual_seed(seed)
    gcn = MetaDenseGCN(data.num_features, 16, data.num_classes, dropout=0.5)
    out["params0"] = np.concatenate([p.detach().numpy().ravel() for p in gcn.parameters()])
    optimizer = torch.optim.Adam([{"params": gcn.layer_in.parameters(), "weight_decay": 5e-4},
                                  {"params": gcn.layer_out.parameters()}], lr=0.01)
    stopper = EarlyStopping(patience)
    rows = []
    gcn.train()
    for epoch in range(epochs):
        optimizer.zero_grad()
        gcn.train()
        o = gcn(data.x, data.dense_adj)
        loss = F.nll_loss(o[data.train_mask], data.y[data.train_mask])
        acc = accuracy(o[data.train_mask], data.y[data.train_mask])
        loss.backward()
        optimizer.step()
        m = evaluate(gcn, data)
        rows.append([loss.item(), acc, m["val.loss"], m["val.accuracy"], m["test.loss"], m["test.accuracy"]])
        stopper.update(m["val.loss"], model=gcn)
        if stopper.abort:
            break
    gcn.load_state_dict(stopper.best_model_state_dict())
    res = evaluate(gcn, data)
    out["seed"] = np.int64(seed)
    out["rows"] = np.array(rows)   # per epoch: train loss, train acc, val loss, val acc, test loss, test acc
    out["final"] = np.array([res["val.loss"], res["val.accuracy"], res["test.loss"], res["test.accuracy"]])
    out["params_final"] = np.concatenate([p.detach().numpy().ravel() for p in gcn.parameters()])
    out["forward_draws"] = np.int64(rnd.forward_counter)


def g_pretrainer(out, n=150, seed=23, patience=20, max_epochs=30):
    """θ pre-training (src/trainers/pretrainer.py): the reference's own
    Pretrainer.train / train_step / evaluate on a BernoulliGraphModel.

    Only __init__ is bypassed: it calls torch_geometric's GAE.split_edges,
    which is absent here.  The split is this repository's restatement
    (ldsgnn.trainers.pretrainer.split_edges, seeded generator) and is stored,
    so the product runs on the identical split; train_adj is filled the way
    src/utils/graph.py:80-116 to_dense_adj fills it (batch None).  θ₀ mixes
    interior values with entries at and beyond the clamp bounds (0, 1, <0, >1)."""
    import src.trainers.pretrainer as pre_mod
    from src.models.graph import BernoulliGraphModel
    from src.utils.early_stopping import EarlyStopping
    from src.utils.graph import triu_values_to_symmetric_matrix
    import torch.nn.functional as F
    sys.path.insert(0, os.path.join(ROOT, "lds-gnn_amd"))
    from ldsgnn.trainers.pretrainer import split_edges
    g =torch.Generator().manual_seed(seed)
    upper = (torch.rand(n, n, generator=g) < 0.06).triu(1)
    adj = (upper | upper.t()).float()
    split = split_edges(adj, generator=torch.Generator().manual_seed(seed + 1))
    tri = n * (n + 1) // 2
    theta0 = torch.rand(tri, generator=g) * 0.8 + 0.1
    special = torch.randperm(tri, generator=g)[:40]
    theta0[special[:10]] = 0.0
    theta0[special[10:20]] = 1.0
    theta0[special[20:30]] = -0.25
    theta0[special[30:40]] = 1.5
    model = BernoulliGraphModel(triu_values_to_symmetric_matrix_raw(theta0, n))
    with torch.no_grad():
        model.probs.copy_(theta0)  # keep the out-of-range entries (the init matrix path would clamp them)
    p = object.__new__(pre_mod.Pretrainer)
    p.model = model
    p.opt = pre_mod.Pretrainer.optimizer(model, lr=0.01, optimizer="adam")
    p.device = torch.device("cpu")

    class _Split:
        pass
    p.data = _Split()
    for k_ref, k in (("train_pos_edge_index", "train_pos"), ("val_pos_edge_index", "val_pos"),
                     ("val_neg_edge_index", "val_neg"), ("test_pos_edge_index", "test_pos"),
                     ("test_neg_edge_index", "test_neg")):
        setattr(p.data, k_ref, split[k])
    train_adj = torch.zeros(n, n)
    train_adj[split["train_pos"][0], split["train_pos"][1]] = 1
    p.train_adj = train_adj
    p.early_stopper = EarlyStopping(patience=patience, max_epochs=max_epochs)
    thetas, losses, vals = [], [], []
    real_bce = F.binary_cross_entropy

    def bce(*a, **k):
        loss = real_bce(*a, **k)
        losses.append(loss.item())
        return loss
    real_step = pre_mod.Pretrainer.train_step

    def step(self, epoch):
        real_step(self, epoch)
        thetas.append(self.model.probs.detach().clone().numpy())
        vals.append([self.evaluate(self.data.val_pos_edge_index, self.data.val_neg_edge_index)[m]
                     for m in ("auc", "average_precision")])
    pre_mod.F = types.SimpleNamespace(binary_cross_entropy=bce)
    pre_mod.Pretrainer.train_step = step
    try:
        res = p.train()
    finally:
        pre_mod.F = F
        pre_mod.Pretrainer.train_step = real_step
    for k, v in split.items():
        out[f"split_{k}"] = v.numpy()
    out["n"] = np.int64(n)
    out["theta0"] = theta0.numpy()
    out["thetas"] = np.stack(thetas)           # θ after every epoch
    out["losses"] = np.array(losses)           # weighted BCE of every epoch (before its step)
    out["val"] = np.array(vals)                # val AUC, AP after every epoch
    out["test"] = np.array([res["auc"], res["average_precision"]])
    out["theta_final"] = p.model.probs.detach().numpy()
    out["patience"] = np.int64(patience)
    out["max_epochs"] = np.int64(max_epochs)


def triu_values_to_symmetric_matrix_raw(theta, n):
    """Symmetric n × n matrix holding θ unclamped (BernoulliGraphModel's init
    matrix; the golden copies θ₀ into probs afterwards anyway)."""
    m = torch.zeros(n, n)
    iu = torch.triu_indices(n, n)
    m[iu[0], iu[1]] = theta
    return torch.maximum(m, m.t())


def main():
    install_stubs()
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    jobs = [("graph_math", g_graph_math), ("sampling_native", g_sampling_native),
            ("gcn_forward", g_gcn_forward), ("adam_first_order", g_adam_first_order),
            ("bilevel_small", g_bilevel),
            ("bilevel_nodrop", lambda o: g_bilevel(o, n=64, f_in=16, classes=3, seed=12, dropout=0.0)),
            ("hypergrad_cora", g_hypergrad_cora), ("conditioning_probe", g_conditioning_probe),
            ("knn_cora", g_knn_cora), ("hypergrad_cora_real", g_hypergrad_cora_real),
            ("hypergrad_cora_real_probe", g_hypergrad_cora_real_probe),
            ("hypergrad_citeseer_s16", g_hypergrad_citeseer_s16),
            ("hypergrad_citeseer_s16_probe", g_hypergrad_citeseer_s16_probe), ("gcn_fixed_cora", g_gcn_fixed_cora),
            ("pretrainer", g_pretrainer), ("hypergrad_cora_wellcond", g_hypergrad_cora_wellcond),
            ("graph_models", g_graph_models), ("hypergrad_citeseer_s16_wellcond", g_hypergrad_citeseer_s16_wellcond)]
    only = set(sys.argv[1:])
    for name, fn in jobs:
        if only and name not in only:
            continue
        out = {}
        fn(out)
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **out)
        print(f"wrote {path} ({os.path.getsize(path) / 1024:.1f} KiB)")


if __name__ == "__main__":
    main()
