"""TEST INFRASTRUCTURE — CPU oracle, never shipped, never on the product path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
anything under oracle/.  The product (lds-gnn_amd/ldsgnn) must not.

A dense PyTorch-CPU (fp32) restatement of the reference's LDS bilevel hot path,
op for op, so that autograd on it reproduces the reference's gradients,
including the double-backward through the differentiable Adam steps:

  θ -> P        triu_values_to_symmetric_matrix   src/utils/graph.py:166-181
  P -> A        sample_graph (NONE, undirected)   src/models/sampling.py:47-85
  A -> Â        normalize_adjacency_matrix        src/utils/graph.py:123-153
  GCN           MetaDenseGCN.forward              src/models/gcn.py:23-34,
                MetaDenseGraphConvolution         src/models/layers.py:30-44
  inner step    InnerProblemTrainer.train_step    src/trainers/inner.py:55-74
                higher.DifferentiableAdam (restated below, see its docstring)
  detach        InnerProblemTrainer.detach        src/trainers/inner.py:98-125
  hyper step    OuterProblemTrainer.train_step    src/trainers/outer.py:57-87
  loop          BilevelProblemRunner.train        src/trainers/bilevel.py:34-126
  eval          empirical_mean_loss               src/utils/evaluation.py:51-84
  early stop    EarlyStopping.update              src/utils/early_stopping.py:19-36

Randomness: the reference's torch-RNG draws are replaced by the keyed Philox
map of oracle/philox.py with the product's (tag, counter) schedule
(ldsgnn/rng.py), or by injected uniforms, so the same edge sets and dropout
masks reach both sides.  Pinned against goldens produced by the reference code
itself (tests/golden/make_golden.py; tests/test_oracle_golden.py).
"""
from __future__ import annotations

import math
from collections import OrderedDict
from typing import Callable, Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

from . import philox

# ----------------------------------------------------------------------------
# graph math (src/utils/graph.py)
# ----------------------------------------------------------------------------


def to_undirected(adj: torch.Tensor, from_triu_only: bool = False) -> torch.Tensor:
    """src/utils/graph.py:27-38"""
    if not from_triu_only:
        return torch.max(adj, adj.t())
    triu = adj.triu(1)
    return triu + triu.t() + torch.diag(adj.diag())


def get_triu_values(adj: torch.Tensor) -> torch.Tensor:
    """src/utils/graph.py:41-45"""
    n = adj.size(0)
    idx = torch.triu_indices(n, n)
    return adj[idx[0], idx[1]]


def num_nodes_from_triu_shape(n_triu_values: int) -> int:
    """src/utils/graph.py:184-192 (same integer arithmetic)."""
    return int(0.5 * math.sqrt((8 * n_triu_values + 1) - 1))


def triu_values_to_symmetric_matrix(triu_values: torch.Tensor) -> torch.Tensor:
    """src/utils/graph.py:166-181"""
    n = num_nodes_from_triu_shape(triu_values.size(0))
    idx = torch.triu_indices(n, n)
    adj = torch.zeros((n, n), dtype=triu_values.dtype)
    adj[idx[0], idx[1]] = triu_values
    adj = to_undirected(adj, from_triu_only=True)
    return adj.clamp(0.0, 1.0)


def add_self_loops(adj: torch.Tensor) -> torch.Tensor:
    """src/utils/graph.py:123-133 — diagonal SET to 1 (its gradient is 0)."""
    c = adj.clone()
    c.fill_diagonal_(1.0)
    return c


def normalize_adjacency_matrix(dense_adj: torch.Tensor) -> torch.Tensor:
    """src/utils/graph.py:136-153"""
    a = add_self_loops(dense_adj)
    deg = a.sum(dim=1)
    inv_sqrt = 1.0 / deg.sqrt()
    d = torch.diag(inv_sqrt)
    return d @ a @ d


def straight_through_estimator(sample: torch.Tensor, parameters: torch.Tensor) -> torch.Tensor:
    """src/models/sampling.py:82-85"""
    return (sample - parameters).detach() + parameters


def sample_graph(edge_probs: torch.Tensor, u: torch.Tensor) -> torch.Tensor:
    """src/models/sampling.py:47-79 with undirected=True, NONE, dense=False.

    `Bernoulli(probs=P).sample()` is `u < P` for u ~ U[0,1) drawn row-major over
    the full N×N matrix (checked bit-exact against torch.bernoulli under the
    same generator in tests/golden); `u` is that N×N draw.
    """
    sample = (u < edge_probs).to(edge_probs.dtype)
    sample = to_undirected(sample, from_triu_only=True)
    return straight_through_estimator(sample, edge_probs)


def graph_uniforms(n: int, seed: int, counter: int, replica: int = 0) -> torch.Tensor:
    """The N×N uniforms the product's sampler uses for draw `counter`."""
    u = philox.uniform(seed, philox.tag_for(philox.TAG_GRAPH, replica), counter, n, n)
    return torch.from_numpy(u)


def dropout(x: torch.Tensor, p: float, training: bool, u: Optional[torch.Tensor]) -> torch.Tensor:
    """F.dropout (src/models/gcn.py:27,29) with the keep decision u < 1 - p."""
    if not training or p == 0.0:
        return x
    keep = np.float32(1.0) - np.float32(p)
    scale = np.float32(1.0) / keep
    mask = (u < float(keep)).to(x.dtype) * float(scale)
    return x * mask


def dropout_uniforms(rows: int, cols: int, seed: int, kind: int, counter: int,
                     replica: int = 0) -> torch.Tensor:
    return torch.from_numpy(philox.uniform(seed, philox.tag_for(kind, replica), counter, rows, cols))


# ----------------------------------------------------------------------------
# GCN (src/models/gcn.py, src/models/layers.py)
# ----------------------------------------------------------------------------

PARAM_NAMES = ("layer_in.fc.weight", "layer_in.fc.bias", "layer_out.fc.weight", "layer_out.fc.bias")


def init_params(in_features: int, hidden: int, out_features: int,
                generator: Optional[torch.Generator] = None) -> "OrderedDict[str, torch.Tensor]":
    """reset_weights (src/models/layers.py:38-40): xavier_uniform_ W, zero b —
    drawn in the order layer_in then layer_out (torch's global CPU generator
    when `generator` is None, exactly as the reference consumes it)."""
    p = OrderedDict()
    for name, (fo, fi) in (("layer_in", (hidden, in_features)), ("layer_out", (out_features, hidden))):
        w = torch.empty(fo, fi)
        with torch.no_grad():
            if generator is None:
                torch.nn.init.xavier_uniform_(w)
            else:
                a = math.sqrt(3.0) * math.sqrt(2.0 / float(fi + fo))
                w.uniform_(-a, a, generator=generator)
        p[f"{name}.fc.weight"] = w
        p[f"{name}.fc.bias"] = torch.zeros(fo)
    return p


def reference_construction_params(in_features: int, hidden: int, out_features: int):
    """MetaDenseGCN.__init__'s draws (src/models/gcn.py:11-17): each
    MetaLinear is an nn.Linear (kaiming weight + uniform bias draws), then
    reset_weights (xavier) — layer_in then layer_out, global CPU generator."""
    p = OrderedDict()
    for name, (fi, fo) in (("layer_in", (in_features, hidden)), ("layer_out", (hidden, out_features))):
        lin = torch.nn.Linear(fi, fo)
        w = torch.nn.init.xavier_uniform_(lin.weight.detach().clone())
        p[f"{name}.fc.weight"] = w
        p[f"{name}.fc.bias"] = torch.zeros(fo)
    return p


def gcn_forward(x: torch.Tensor, adj: torch.Tensor, params, dropout_p: float, training: bool,
                u_x: Optional[torch.Tensor] = None, u_h: Optional[torch.Tensor] = None,
                normalize_adj: bool = True) -> torch.Tensor:
    """MetaDenseGCN.forward (src/models/gcn.py:23-34): bias before aggregation."""
    a = normalize_adjacency_matrix(adj) if normalize_adj else adj
    h = dropout(x, dropout_p, training, u_x)
    h = F.linear(h, params["layer_in.fc.weight"], params["layer_in.fc.bias"])
    h = F.relu(torch.mm(a, h))
    h = dropout(h, dropout_p, training, u_h)
    h = F.linear(h, params["layer_out.fc.weight"], params["layer_out.fc.bias"])
    h = torch.mm(a, h)
    return F.log_softmax(h, dim=1)


def accuracy(pred: torch.Tensor, labels: torch.Tensor) -> float:
    """src/utils/evaluation.py:15-22"""
    return (torch.argmax(pred, dim=-1) == labels).float().mean().item()


# ----------------------------------------------------------------------------
# higher.DifferentiableAdam, restated
# ----------------------------------------------------------------------------


class DifferentiableAdam:
    """Restatement of `higher.optim.DifferentiableAdam` (facebookresearch/higher,
    unpinned git HEAD per scripts/install.sh:3-4; not vendored in the reference),
    as called from src/trainers/inner.py:48-50,71:

        g = autograd.grad(loss, params, create_graph=True)
        g = g + weight_decay * p                     (group 0 only: 5e-4)
        step += 1; bc1 = 1 - b1**step; bc2 = 1 - b2**step
        m = m * b1 + (1 - b1) * g
        v = v * b2 + (1 - b2) * g * g
        (gradient of v masked to 0 where v == 0 — higher's _maybe_mask hook)
        denom = sqrt(v) / sqrt(bc2) + eps
        p = p - (lr / bc1) * m / denom                (addcdiv)

    `groups` = [(param indices, weight_decay)], one lr / betas / eps.
    """

    def __init__(self, groups: List[Tuple[List[int], float]], lr: float,
                 betas=(0.9, 0.999), eps: float = 1e-8):
        self.groups = groups
        self.lr = lr
        self.betas = betas
        self.eps = eps
        self.state: Dict[int, Dict[str, object]] = {}

    def step(self, loss: torch.Tensor, params: List[torch.Tensor]) -> List[torch.Tensor]:
        grads = torch.autograd.grad(loss, params, create_graph=True, allow_unused=True)
        b1, b2 = self.betas
        new = list(params)
        for idxs, wd in self.groups:
            for i in idxs:
                p, g = params[i], grads[i]
                if g is None:
                    continue
                st = self.state.setdefault(i, {})
                if len(st) == 0:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p.data)
                    st["exp_avg_sq"] = torch.zeros_like(p.data)
                st["step"] += 1
                bc1 = 1 - b1 ** st["step"]
                bc2 = 1 - b2 ** st["step"]
                if wd != 0:
                    g = g + (wd * p)
                m = (st["exp_avg"] * b1) + (1 - b1) * g
                v = (st["exp_avg_sq"] * b2) + (1 - b2) * g * g
                mask = v == 0.0
                if v.requires_grad:
                    v.register_hook(lambda grad, mask=mask: grad.masked_fill(mask, 0.0))
                st["exp_avg"], st["exp_avg_sq"] = m, v
                denom = (v.sqrt() / math.sqrt(bc2)) + self.eps
                new[i] = torch.addcdiv(p, m, denom, value=-(self.lr / bc1))
        return new

    def detach_(self) -> None:
        """InnerProblemTrainer.detach_optimizer (src/trainers/inner.py:110-125)."""
        for st in self.state.values():
            for k in ("exp_avg", "exp_avg_sq"):
                st[k] = st[k].detach().requires_grad_()


def copy_detach(params):
    """copy_detach_parameter_dict (src/trainers/inner.py:15-19)."""
    return OrderedDict((k, v.detach().clone().requires_grad_(True)) for k, v in params.items())


# ----------------------------------------------------------------------------
# Early stopping (src/utils/early_stopping.py:19-36)
# ----------------------------------------------------------------------------


class EarlyStopping:
    def __init__(self, patience: int, max_epochs: int = 10000):
        self.abort = False
        self.patience = patience
        self.model_params = None
        self.max_epochs = max_epochs
        self.curr_step = 0
        self.losses: List[float] = []

    def update(self, new_value, model_params=None):
        self.losses.append(new_value)
        if self.curr_step <= self.patience or new_value <= np.mean(self.losses[-(self.patience + 1):-1]):
            if model_params is not None:
                self.model_params = model_params
        else:
            self.abort = True
        if self.curr_step is not None and self.curr_step >= self.max_epochs:
            self.abort = True
        self.curr_step += 1


# ----------------------------------------------------------------------------
# The bilevel problem (src/trainers/{inner,outer,bilevel}.py)
# ----------------------------------------------------------------------------


class Randomness:
    """The product's draw schedule (ldsgnn/rng.py): every graph sample takes the
    next graph counter, every training-mode forward the next forward counter."""

    def __init__(self, seed: int, replica: int = 0, inject_graph: Optional[Callable] = None):
        self.seed = seed
        self.replica = replica
        self.graph_counter = 0
        self.forward_counter = 0
        self.inject_graph = inject_graph

    def graph_u(self, n: int) -> torch.Tensor:
        c = self.graph_counter
        self.graph_counter += 1
        if self.inject_graph is not None:
            return self.inject_graph(c)
        return graph_uniforms(n, self.seed, c, self.replica)

    def forward_u(self, n: int, f_in: int, hidden: int, p: float, training: bool):
        if not training or p == 0.0:
            return None, None
        c = self.forward_counter
        self.forward_counter += 1
        ux = dropout_uniforms(n, f_in, self.seed, philox.TAG_DROP_X, c, self.replica)
        uh = dropout_uniforms(n, hidden, self.seed, philox.TAG_DROP_H, c, self.replica)
        return ux, uh


class LdsProblem:
    """State of one LDS run: θ, GCN params + Adam state, the data."""

    def __init__(self, x, y, train_mask, val_mask, test_mask, opt_mask, theta: torch.Tensor,
                 hidden: int = 16, dropout_p: float = 0.5, gcn_lr: float = 0.01,
                 gcn_wd: float = 5e-4, outer_lr: float = 1.0, lr_decay: Optional[float] = None,
                 rnd: Optional[Randomness] = None, init_generator: Optional[torch.Generator] = None,
                 params: Optional["OrderedDict[str, torch.Tensor]"] = None):
        self.x, self.y = x, y
        self.train_mask, self.val_mask, self.test_mask, self.opt_mask = train_mask, val_mask, test_mask, opt_mask
        self.n, self.f_in = x.shape
        self.c = int(y.max()) + 1
        self.hidden = hidden
        self.dropout_p = dropout_p
        self.gcn_lr, self.gcn_wd = gcn_lr, gcn_wd
        self.theta = theta.clone().requires_grad_(True)
        self.outer_lr = outer_lr
        self.lr_decay = lr_decay
        self.rnd = rnd or Randomness(0)
        self.init_generator = init_generator
        if params is None:
            self.reset_weights()
        else:
            self.params = OrderedDict((k, v.detach().clone().requires_grad_(True)) for k, v in params.items())
        self.reset_optimizer()

    # --- inner (src/trainers/inner.py) ---
    def reset_weights(self):
        self.params = init_params(self.f_in, self.hidden, self.c, self.init_generator)
        for v in self.params.values():
            v.requires_grad_(True)

    def reset_optimizer(self):
        self.opt = DifferentiableAdam([([0, 1], self.gcn_wd), ([2, 3], 0.0)], lr=self.gcn_lr)

    def sample(self) -> torch.Tensor:
        """BernoulliGraphModel.sample (src/models/graph.py:29-32, 66-67)."""
        p = triu_values_to_symmetric_matrix(self.theta)
        return sample_graph(p, self.rnd.graph_u(self.n))

    def forward(self, graph: torch.Tensor, training: bool = True, params=None) -> torch.Tensor:
        ux, uh = self.rnd.forward_u(self.n, self.f_in, self.hidden, self.dropout_p, training)
        return gcn_forward(self.x, graph, params if params is not None else self.params,
                           self.dropout_p, training, ux, uh)

    def inner_step(self, graph: torch.Tensor) -> Tuple[float, float]:
        pred = self.forward(graph, True)
        m = self.train_mask
        loss = F.nll_loss(pred[m], self.y[m])
        acc = accuracy(pred[m], self.y[m])
        new = self.opt.step(loss, list(self.params.values()))
        self.params = OrderedDict(zip(self.params.keys(), new))
        return loss.item(), acc

    def detach(self):
        self.params = copy_detach(self.params)
        self.opt.detach_()

    # --- outer (src/trainers/outer.py:57-87) ---
    def hyper_step(self) -> Tuple[float, float, torch.Tensor]:
        """src/trainers/outer.py:57-87 + the detaches of bilevel.py:109-114."""
        loss, acc, grad = self.hyper_grad()
        self.apply_hyper_update(grad)
        return loss, acc, grad

    def hyper_grad(self) -> Tuple[float, float, torch.Tensor]:
        """The outer loss.backward of a hyper step: (loss, acc, dθ); θ unchanged."""
        if self.theta.grad is not None:
            self.theta.grad = None
        graph = self.sample()
        pred = self.forward(graph, True)
        m = self.opt_mask
        loss = F.nll_loss(pred[m], self.y[m])
        acc = accuracy(pred[m], self.y[m])
        loss.backward(retain_graph=True)
        return loss.item(), acc, self.theta.grad.detach().clone()

    def apply_hyper_update(self, grad: torch.Tensor) -> None:
        """SGD (no momentum) → StepLR → clamp (project_parameters), then detach."""
        with torch.no_grad():
            self.theta.add_(grad, alpha=-self.outer_lr)                # SGD, no momentum
            if self.lr_decay is not None:
                self.outer_lr = self.outer_lr * self.lr_decay          # StepLR(step_size=1)
            self.theta.clamp_(0.0, 1.0)                                # project_parameters
        self.detach()

    def empirical_mean_loss(self, n_samples: int, params=None):
        """src/utils/evaluation.py:51-84"""
        vl, va, tl, ta = [], [], [], []
        with torch.no_grad():
            for _ in range(n_samples):
                g = self.sample()
                pred = self.forward(g, False, params)
                vl.append(F.nll_loss(pred[self.val_mask], self.y[self.val_mask]).item())
                va.append(accuracy(pred[self.val_mask], self.y[self.val_mask]))
                tl.append(F.nll_loss(pred[self.test_mask], self.y[self.test_mask]).item())
                ta.append(accuracy(pred[self.test_mask], self.y[self.test_mask]))
        return (float(np.mean(vl)), float(np.mean(va))), (float(np.mean(tl)), float(np.mean(ta)))

    # --- loop (src/trainers/bilevel.py:34-107) ---
    def train(self, patience: int, hyper_gradient_interval: int, inner_loop_max_epochs: int = 400,
              outer_loop_max_epochs: int = 400, n_samples_empirical_mean: int = 16,
              log: Optional[List] = None):
        outer_stop = EarlyStopping(patience, outer_loop_max_epochs)
        step = 0
        while not outer_stop.abort:
            inner_stop = EarlyStopping(patience, inner_loop_max_epochs)
            self.reset_weights()
            self.reset_optimizer()
            while not inner_stop.abort:
                loss, acc = self.inner_step(self.sample())
                inner_stop.update(loss, model_params=copy_detach(self.params))
                if log is not None:
                    log.append(("inner", step, loss, acc))
                if hyper_gradient_interval == 0 or step % hyper_gradient_interval == 0:
                    ol, oa, _ = self.hyper_step()
                    if log is not None:
                        log.append(("outer", step, ol, oa))
                step += 1
            best = inner_stop.model_params
            (vl, va), (tl, ta) = self.empirical_mean_loss(n_samples_empirical_mean, best)
            if log is not None:
                log.append(("empirical", step, vl, va, tl, ta))
            # the reference stores outer_trainer.model.state_dict(): live views
            # of θ, not copies (src/trainers/bilevel.py:96-98) — kept as such.
            outer_stop.update(vl, model_params=[best, self.theta.detach()])
        self.best_params, self.best_theta = outer_stop.model_params
        self.n_samples_empirical_mean = n_samples_empirical_mean
        return step

    def evaluate(self):
        """BilevelProblemRunner.evaluate (src/trainers/bilevel.py:128-145)."""
        with torch.no_grad():
            self.theta.copy_(self.best_theta)
        (vl, va), (tl, ta) = self.empirical_mean_loss(self.n_samples_empirical_mean, self.best_params)
        return {"loss.val.final": vl, "acc.val.final": va, "loss.test.final": tl, "acc.test.final": ta}

    def run_steps(self, inner_steps: int, hyper_gradient_interval: int):
        """Fixed-count inner loop with hyper steps every τ (benchmark protocol,
        SURVEY §8(d): early stopping disabled)."""
        out = []
        for step in range(inner_steps):
            loss, acc = self.inner_step(self.sample())
            out.append(loss)
            if hyper_gradient_interval == 0 or step % hyper_gradient_interval == 0:
                self.hyper_step()
        return out


def replica_hyper_step(problems: List["LdsProblem"]) -> Tuple[List[Tuple[float, float]], torch.Tensor]:
    """One hyper step of S Monte-Carlo replicas (not in the
    reference, which runs S = 1): every replica — its own graph / dropout
    stream (Randomness replica b), GCN weights and Adam state, the same θ —
    computes its hypergradient; the mean over replicas (what an all-reduce
    SUM / S gives) updates every replica's θ identically.  S = 1 is exactly
    LdsProblem.hyper_step."""
    res = [p.hyper_grad() for p in problems]
    g = res[0][2].clone()
    for r in res[1:]:
        g += r[2]
    g /= len(problems)
    for p in problems:
        p.apply_hyper_update(g)
    return [(r[0], r[1]) for r in res], g


def pretrain_epoch_dense(theta: torch.Tensor, train_adj: torch.Tensor, optimizer: torch.optim.Optimizer) -> float:
    """One Pretrainer.train_step (src/trainers/pretrainer.py:68-81) restated
    densely: P = triu_values_to_symmetric_matrix(θ), weighted BCE against the
    training adjacency, backward, optimizer.step().  θ: the Parameter the
    optimizer holds."""
    optimizer.zero_grad()
    p = triu_values_to_symmetric_matrix(theta)
    pos_weight = (train_adj.numel() - train_adj.sum().item()) / train_adj.sum().item()
    weight = (train_adj * (pos_weight - 1)) + 1.0
    loss = F.binary_cross_entropy(p, train_adj, weight=weight)
    loss.backward()
    optimizer.step()
    return loss.item()


class FixedGcnTraining:
    """BASELINE config 1: the reference's fixed-graph GCN training loop
    (src/scripts/gcn.py:56-99) restated — MetaDenseGCN on the constant given
    adjacency (normalised densely every forward, src/models/gcn.py:24-25),
    torch.optim.Adam with the two parameter groups of gcn.py:62-67 (weight
    decay on layer_in only), and per epoch: train forward (dropout from the
    keyed stream), NLL on the train mask, backward, step, then evaluate()
    (src/utils/evaluation.py:25-48: eval forward, val/test loss and accuracy)
    and EarlyStopping on val.loss (src/utils/early_stopping.py:19-36)."""

    def __init__(self, x, y, adj, train_mask, val_mask, test_mask, hidden: int = 16, dropout_p: float = 0.5,
                 lr: float = 0.01, wd: float = 5e-4, rnd: Optional[Randomness] = None,
                 init_generator: Optional[torch.Generator] = None, params=None, patience: int = 10):
        self.x, self.y, self.adj = x, y, adj
        self.train_mask, self.val_mask, self.test_mask = train_mask, val_mask, test_mask
        self.n, self.f_in = x.shape
        self.c = int(y.max()) + 1
        self.hidden, self.dropout_p = hidden, dropout_p
        self.rnd = rnd or Randomness(0)
        if params is None:
            params = init_params(self.f_in, hidden, self.c, init_generator)
        self.params = OrderedDict((k, v.detach().clone().requires_grad_(True)) for k, v in params.items())
        ps = list(self.params.values())
        self.opt = torch.optim.Adam([{"params": ps[:2], "weight_decay": wd}, {"params": ps[2:]}], lr=lr)
        self.stopper = EarlyStopping(patience)

    def forward(self, training: bool) -> torch.Tensor:
        ux, uh = self.rnd.forward_u(self.n, self.f_in, self.hidden, self.dropout_p, training)
        return gcn_forward(self.x, self.adj, self.params, self.dropout_p, training, ux, uh)

    def evaluate(self) -> Dict[str, float]:
        with torch.no_grad():
            out = self.forward(False)
            vm, tm = self.val_mask, self.test_mask
            return {"val.accuracy": accuracy(out[vm], self.y[vm]),
                    "val.loss": F.nll_loss(out[vm], self.y[vm]).item(),
                    "test.accuracy": accuracy(out[tm], self.y[tm]),
                    "test.loss": F.nll_loss(out[tm], self.y[tm]).item()}

    def epoch(self) -> Tuple[float, float, Dict[str, float]]:
        """One iteration of src/scripts/gcn.py:75-91; returns (train loss,
        train acc, evaluate()) and updates the early stopper."""
        self.opt.zero_grad()
        out = self.forward(True)
        m = self.train_mask
        loss = F.nll_loss(out[m], self.y[m])
        acc = accuracy(out[m], self.y[m])
        loss.backward()
        self.opt.step()
        metrics = self.evaluate()
        self.stopper.update(metrics["val.loss"])
        return loss.item(), acc, metrics
