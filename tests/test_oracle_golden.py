"""Pin the CPU oracle against golden vectors produced by the reference code
itself (tests/golden/make_golden.py) and against the reference's own
known-answer tests.  CPU only."""
import os
from collections import OrderedDict

import numpy as np
import pytest
import torch

from oracle import lds_oracle as O
from oracle import philox

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def gold(name):
    return np.load(os.path.join(GOLD, f"{name}.npz"))


def prob_from(g):
    t = lambda k: torch.from_numpy(g["prob_" + k])  # noqa: E731
    return dict(x=t("x"), y=t("y"), train=t("train"), val=t("val"), opt=t("opt"), test=t("test"),
                adj=t("adj"))


# --- reference known-answer tests (tst/) ------------------------------------

def test_kat_triu_values_to_symmetric_matrix():
    """tst/utils/test_graph.py:213-221"""
    p = O.triu_values_to_symmetric_matrix(torch.as_tensor([0.1, 0.2, 0.3, 0.4, 0.5, 0.6]))
    assert p.equal(torch.as_tensor([[0.1, 0.2, 0.3], [0.2, 0.4, 0.5], [0.3, 0.5, 0.6]]))


def test_kat_to_undirected_triu():
    """tst/utils/test_graph.py:43-52"""
    m = torch.zeros(10, 10)
    m[:, 1] = 1.0
    e = torch.zeros(10, 10)
    e[0, 1] = e[1, 1] = e[1, 0] = 1.0
    assert O.to_undirected(m, from_triu_only=True).equal(e)


@pytest.mark.parametrize("nodes", [10, 100, 1000, 2000, 500000])
def test_kat_num_nodes_from_triu_shape(nodes):
    """tst/utils/test_graph.py:232-235"""
    assert O.num_nodes_from_triu_shape(int(nodes ** 2 / 2 + nodes / 2)) == nodes


def test_kat_self_loop_gradient_is_zero_on_diagonal():
    """tst/utils/test_graph.py:169-178"""
    m = torch.rand(100, 100).requires_grad_(True)
    O.add_self_loops(m).sum().backward()
    nz = m.grad.nonzero()
    assert (nz[:, 0] != nz[:, 1]).all() and nz.size(0) == 100 * 99


def test_kat_deterministic_sampling():
    """tst/models/test_sampling.py:149-153: θ ∈ {0,1} -> A = 1 - I."""
    n = 20
    p = torch.ones(n, n).triu(1)
    a = O.sample_graph(p, torch.rand(n, n))
    assert a.equal(torch.ones(n, n) - torch.eye(n))


def test_kat_early_stopping():
    """tst/utils/test_early_stopping.py:6-40"""
    def run(patience, max_epochs, seq):
        es = O.EarlyStopping(patience=patience, max_epochs=max_epochs)
        for v in seq:
            es.update(v)
            if es.abort:
                return es.curr_step
    assert run(1, 100, [-a for a in range(1000)]) == 101
    assert run(20, 100, [42.0 + a for a in range(1000)]) == 22
    assert run(34, 1000, [42.0 - a if a < 500 else 42.0 + a for a in range(1000)]) == 501


def test_kat_accuracy():
    """tst/utils/test_evaluation.py:12-18"""
    pred = torch.as_tensor([[0.1, 0.9, 0.0], [0.1, 0.9, 0.0], [0.0, 0.0, 1.0]])
    assert np.isclose(O.accuracy(pred, torch.as_tensor([1, 0, 2])), 2.0 / 3.0)


# --- goldens from the reference code ----------------------------------------

def test_graph_math_golden():
    g = gold("graph_math")
    assert np.array_equal(O.triu_values_to_symmetric_matrix(torch.from_numpy(g["theta8"])).numpy(), g["p8"])
    assert np.allclose(O.normalize_adjacency_matrix(torch.from_numpy(g["adj16"])).numpy(), g["norm16"],
                       rtol=1e-6, atol=1e-7)


def test_theta_gradient_golden_and_closed_form():
    """θ-gradient through P -> STE sample -> normalisation: the oracle's
    autograd AND the closed form the HIP kernel implements
    against the reference's autograd."""
    g = gold("graph_math")
    n = 30
    theta = torch.from_numpy(g["theta30"]).requires_grad_(True)
    w = torch.from_numpy(g["w30"])
    u = O.graph_uniforms(n, int(g["seed30"]), 0)
    a = O.sample_graph(O.triu_values_to_symmetric_matrix(theta), u)
    assert np.array_equal(a.detach().numpy(), g["sample30"])
    (w * O.normalize_adjacency_matrix(a)).sum().backward()
    assert np.allclose(theta.grad.numpy(), g["grad30"], rtol=1e-5, atol=1e-7)
    # closed form: dθ_ij = s_i s_j (M_ij + M_ji) + r_i + r_j, dθ_ii = 0,
    # r_i = -1/2 s_i^3 sum_k (M_ik + M_ki) Ã_ik s_k, M = dL/dÂ = w
    at = a.detach().double().clone()
    at.fill_diagonal_(1.0)
    s = 1.0 / at.sum(1).sqrt()
    m = w.double()
    msym = m + m.t()
    r = -0.5 * s ** 3 * ((msym * at) @ s)
    full = s[:, None] * s[None, :] * msym + r[:, None] + r[None, :]
    iu = torch.triu_indices(n, n)
    closed = full[iu[0], iu[1]]
    closed[iu[0] == iu[1]] = 0.0
    assert np.allclose(closed.numpy(), g["grad30"], rtol=1e-5, atol=1e-6)


def test_sampling_native_rng_golden():
    """u < P with u = torch.rand under the same seed == Bernoulli(P).sample()."""
    g = gold("sampling_native")
    n = 64
    torch.manual_seed(77)
    u = torch.rand(n, n)
    assert np.array_equal(u.numpy(), g["u"])
    p = O.triu_values_to_symmetric_matrix(torch.from_numpy(g["theta"]))
    assert np.array_equal(O.sample_graph(p, u).detach().numpy(), g["sample"])


def test_gcn_forward_golden():
    g = gold("gcn_forward")
    pr = prob_from(g)
    n, f_in = pr["x"].shape
    seed = int(g["seed"])
    flat = torch.from_numpy(g["params"])
    shapes = [(16, f_in), (16,), (5, 16), (5,)]
    params, off = OrderedDict(), 0
    for name, shp in zip(O.PARAM_NAMES, shapes):
        k = int(np.prod(shp))
        params[name] = flat[off:off + k].reshape(shp)
        off += k
    theta = torch.from_numpy(g["theta"])
    a = O.sample_graph(O.triu_values_to_symmetric_matrix(theta), O.graph_uniforms(n, seed, 0))
    ux = O.dropout_uniforms(n, f_in, seed, philox.TAG_DROP_X, 0)
    uh = O.dropout_uniforms(n, 16, seed, philox.TAG_DROP_H, 0)
    out = O.gcn_forward(pr["x"], a, params, 0.5, True, ux, uh)
    assert np.allclose(out.detach().numpy(), g["train_logp"], rtol=1e-5, atol=1e-6)
    out = O.gcn_forward(pr["x"], a, params, 0.5, False)
    assert np.allclose(out.detach().numpy(), g["eval_logp"], rtol=1e-5, atol=1e-6)


def test_differentiable_adam_matches_torch_adam_first_order():
    """higher's update restated == torch.optim.Adam values (golden)."""
    g = gold("adam_first_order")
    pr = prob_from(g)
    f_in = pr["x"].shape[1]
    flat = torch.from_numpy(g["params0"])
    shapes = [(16, f_in), (16,), (4, 16), (4,)]
    params, off = OrderedDict(), 0
    for name, shp in zip(O.PARAM_NAMES, shapes):
        k = int(np.prod(shp))
        params[name] = flat[off:off + k].reshape(shp).clone().requires_grad_(True)
        off += k
    opt = O.DifferentiableAdam([([0, 1], 5e-4), ([2, 3], 0.0)], lr=0.01)
    plist = list(params.values())
    for step in range(5):
        out = O.gcn_forward(pr["x"], pr["adj"], OrderedDict(zip(O.PARAM_NAMES, plist)), 0.0, True)
        loss = torch.nn.functional.nll_loss(out[pr["train"]], pr["y"][pr["train"]])
        plist = opt.step(loss, plist)
        got = np.concatenate([p.detach().numpy().ravel() for p in plist])
        assert np.allclose(got, g["trajectory"][step], rtol=1e-5, atol=1e-6), step


def run_oracle_bilevel(g):
    pr = prob_from(g)
    seed = int(g["seed"])
    n, f_in = pr["x"].shape
    c = int(pr["y"].max()) + 1
    torch.manual_seed(seed)
    params = O.reference_construction_params(f_in, 16, c)
    prob = O.LdsProblem(pr["x"], pr["y"], pr["train"], pr["val"], pr["test"], pr["opt"],
                        O.get_triu_values(pr["adj"]), hidden=16, dropout_p=float(g["dropout"]),
                        gcn_lr=0.01, gcn_wd=5e-4, outer_lr=0.1, lr_decay=0.99,
                        rnd=O.Randomness(seed), params=params)
    log, grads = [], []
    orig = prob.hyper_step

    def spy():
        r = orig()
        grads.append(r[2].numpy())
        return r

    prob.hyper_step = spy
    prob.train(patience=3, hyper_gradient_interval=5, inner_loop_max_epochs=12, outer_loop_max_epochs=2, log=log)
    final = prob.evaluate()
    return prob, log, grads, final


@pytest.mark.parametrize("name", ["bilevel_small", "bilevel_nodrop"])
def test_bilevel_training_golden(name):
    """The whole reference training loop (early stopping, τ=5 hyper steps,
    16-sample empirical evaluation, final evaluate) reproduced by the oracle."""
    g = gold(name)
    prob, log, grads, final = run_oracle_bilevel(g)
    names, vals = g["log_names"], g["log_values"]
    ref_train = vals[names == "loss.train"]
    ref_outer = vals[names == "loss.outer"]
    ref_emp = vals[names == "loss.val.empirical"]
    ref_emp_test_acc = vals[names == "acc.test.empirical"]
    got_train = np.array([r[2] for r in log if r[0] == "inner"])
    got_outer = np.array([r[2] for r in log if r[0] == "outer"])
    got_emp = np.array([r[2] for r in log if r[0] == "empirical"])
    got_emp_test_acc = np.array([r[5] for r in log if r[0] == "empirical"])
    assert got_train.shape == ref_train.shape and got_outer.shape == ref_outer.shape
    assert np.allclose(got_train, ref_train, rtol=1e-5, atol=1e-6)
    assert np.allclose(got_outer, ref_outer, rtol=1e-5, atol=1e-6)
    assert np.allclose(got_emp, ref_emp, rtol=1e-5, atol=1e-6)
    assert np.allclose(got_emp_test_acc, ref_emp_test_acc, atol=1e-6)
    assert len(grads) == len(g["theta_grads"])
    for a, b in zip(grads, g["theta_grads"]):
        assert np.allclose(a, b, rtol=1e-4, atol=1e-6)
    assert np.allclose(prob.theta.detach().numpy(), g["theta_final"], rtol=1e-5, atol=1e-6)
    assert np.allclose([final["loss.val.final"], final["acc.val.final"], final["loss.test.final"],
                        final["acc.test.final"]], g["final"], rtol=1e-5, atol=1e-6)
    assert prob.rnd.graph_counter == int(g["graph_draws"])
    assert prob.rnd.forward_counter == int(g["forward_draws"])


class _Data:
    pass


def cora_golden_problem(g):
    """The Cora-shaped problem exactly as the golden stored it (X as CSR, the
    kNN θ₀ as an edge list): nothing recomputed, so no machine dependence."""
    n, f = (int(v) for v in g["x_shape"])
    x = torch.sparse_csr_tensor(torch.from_numpy(g["x_indptr"]), torch.from_numpy(g["x_indices"]).long(),
                                torch.from_numpy(g["x_values"]), size=(n, f)).to_dense()
    adj = torch.zeros(n, n)
    e = torch.from_numpy(g["adj_edges"]).long()
    adj[e[0], e[1]] = 1.0
    adj[e[1], e[0]] = 1.0
    d = _Data()
    d.x, d.dense_adj, d.y = x, adj, torch.from_numpy(g["y"])
    d.train_mask, d.val_mask, d.test_mask = (torch.from_numpy(g[k]) for k in ("train_mask", "val_mask", "test_mask"))
    return d, torch.from_numpy(g["opt_mask"]), int(g["seed"])


@pytest.mark.slow
def test_hypergradient_cora_golden():
    """A τ=5 truncated hypergradient at Cora shape (N=2708, F_in=1433)."""
    g = gold("hypergrad_cora")
    data, opt, seed = cora_golden_problem(g)
    torch.manual_seed(seed)
    params = O.reference_construction_params(data.x.shape[1], 16, 7)
    prob = O.LdsProblem(data.x, data.y, data.train_mask, data.val_mask & ~opt, data.test_mask, opt,
                        O.get_triu_values(data.dense_adj), dropout_p=0.5, outer_lr=0.1, lr_decay=0.99,
                        rnd=O.Randomness(seed), params=params)
    losses, grad = [], None
    for step in range(6):
        losses.append(prob.inner_step(prob.sample())[0])
        if step % 5 == 0:
            grad = prob.hyper_step()[2].double().numpy()
    assert np.allclose(losses, g["inner_losses"], rtol=1e-5, atol=1e-6)
    idx = g["grad_idx"]
    assert np.allclose(grad[idx], g["grad_val"], rtol=1e-4, atol=1e-7)
    assert np.isclose(grad.sum(), g["grad_sum"], rtol=1e-4, atol=1e-6)
    assert np.isclose(np.sqrt((grad ** 2).sum()), g["grad_l2"], rtol=1e-5)
    th = prob.theta.detach().numpy()
    assert np.allclose(th[g["theta_idx"]], g["theta_val"], rtol=1e-5, atol=1e-7)


def test_pretrain_epochs_golden():
    """oracle.pretrain_epoch_dense + torch.optim.Adam against the reference's
    own Pretrainer.train_step (golden `pretrainer`): θ after every epoch and
    the epoch's weighted BCE, bit for bit (the same dense ops in the same
    order on CPU)."""
    g = gold("pretrainer")
    n = int(g["n"])
    tp = torch.from_numpy(g["split_train_pos"])
    train_adj = torch.zeros(n, n)
    train_adj[tp[0], tp[1]] = 1
    theta = torch.nn.Parameter(torch.from_numpy(g["theta0"]).clone())
    opt = torch.optim.Adam([theta], lr=0.01)
    for e in range(g["thetas"].shape[0]):
        loss = O.pretrain_epoch_dense(theta, train_adj, opt)
        assert loss == float(g["losses"][e]), e
        assert np.array_equal(theta.detach().numpy(), g["thetas"][e]), e
