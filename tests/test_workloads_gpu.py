"""The benched path — the fused engine, captured τ-window HIP graph replayed —
at the BASELINE workloads' own sizes, against goldens the REFERENCE code made
(tests/golden/make_golden.py; no oracle in between):

  config 2  real Cora, kNN θ₀ (knn_cora), S = 1: golden hypergrad_cora_real
            (the reference's step-0 hyper step and its τ = 5 window)
  config 3  real Citeseer, θ₀ = given graph, S = 16 replicas batched in one
            engine: golden hypergrad_citeseer_s16 (16 reference runners,
            replica b on the keyed stream of replica b, mean hypergradient);
            its window starts at Adam step 1, so its dθ is held against the
            reference's own rounding probe like config 2's (below)

Tolerances (fp32, north_star 1e-5): losses, θ and weights 1e-5 relative; dθ
entries 1e-5 × max|dθ| (the kernel tests' criterion: an entry is a sum of
terms s_i s_j (M_ij + M_ji) + r_i + r_j that cancel, so its fp32 error scales
with the terms, not with the result — the engine's split-bf16 assembly and
fp32 reductions reorder the reference's dense fp32 sums), and
‖dθ‖₂ 1e-5 relative.

The exception, measured on the reference itself: its hypergradient is
ill-conditioned.  higher's Adam update lr·m̂/(√v̂ + eps) has derivative up to
lr/eps = 10⁶ in g for parameters whose |g| is near eps (and at the first Adam
step the update is ≈ lr·sign(g)), so rounding differences in those gradients
are amplified into dθ and into a few weights.  Golden
hypergrad_cora_real_probe re-runs the REFERENCE with its two matrix products
(aggregation torch.mm, F.linear) summed in fp64 — a pure rounding change — and
moves by: step-0 dθ 5.1e-4 × max|dθ|, window dθ 2.9e-5 × max|dθ|, weights
2.7e-6 absolute.  The engine's deviations sit on the same entries (top-50
error entries ≥ 60 % shared with the probe's, measured 80-98 %) at ≤ 5.2× the
probe's size (measured: 1.7×, 5.2×, 5.1×); the test holds them to 8× the
reference's own movement, and everything the conditioning does not reach
(losses, θ) to 1e-5.
"""
import numpy as np
import pytest
import torch

import ldsgnn
from ldsgnn.data.workloads import load_workload
from ldsgnn.fused import engine_from_trainers
from ldsgnn.models.gcn import MetaDenseGCN
from ldsgnn.models.graph import BernoulliGraphModel
from ldsgnn.trainers.inner import InnerProblemTrainer
from ldsgnn.trainers.outer import OuterProblemTrainer
from tests.conftest import GOLDEN

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-5
GRAD_TOL = 1e-5


def _trainers(workload, g, seed, replica=0, dropout=0.5):
    data = load_workload(workload)
    data.val_mask = torch.from_numpy(g["val_mask"])
    opt = torch.from_numpy(g["opt_mask"]).to(DEV)
    data = data.to(DEV)
    ldsgnn.rng.manual_seed(seed, replica)
    torch.manual_seed(seed)
    gcn = MetaDenseGCN(data.num_features, 16, data.num_classes, dropout=dropout).to(DEV)
    inner = InnerProblemTrainer(gcn, data, lr=0.01, weight_decay=5e-4)
    gm = BernoulliGraphModel(data.dense_adj)
    outer = OuterProblemTrainer(torch.optim.SGD(gm.parameters(), lr=0.1), data, opt, gm, lr_decay=0.99)
    return data, inner, outer, gm


def _check_vec(got, g, key, tol):
    got = got.detach().double().cpu().numpy()
    idx = g["idx"]
    ref = g[key + "_val"].astype(np.float64)
    scale = np.abs(ref).max()
    err = np.abs(got[idx] - ref)
    diag = (key, float(err.max() / scale), float(np.sqrt((err ** 2).sum() / (ref ** 2).sum())), tol)
    assert err.max() <= tol * scale, diag
    assert np.isclose(np.sqrt((got ** 2).sum()), float(g[key + "_l2"]), rtol=max(tol, 1e-5)), diag
    assert np.isclose(got.sum(), float(g[key + "_sum"]), rtol=max(tol, 1e-4), atol=1e-5 * scale), diag


PROBE_FACTOR = 8.0


def _probe_tol(g, p, key):
    """PROBE_FACTOR × how far the reference's own dθ moves under a pure
    rounding change (relative to max|dθ|), at least GRAD_TOL."""
    a, b = g[key + "_val"].astype(np.float64), p[key + "_val"].astype(np.float64)
    return max(GRAD_TOL, PROBE_FACTOR * float(np.abs(a - b).max() / np.abs(a).max()))


def _same_entries_as_probe(got, g, p, key, top=50):
    """The engine's largest deviations fall on the entries the reference's own
    rounding probe moves most (the ill-conditioned ones)."""
    ref = g[key + "_val"].astype(np.float64)
    eg = np.abs(got.detach().double().cpu().numpy()[g["idx"]] - ref)
    ep = np.abs(p[key + "_val"].astype(np.float64) - ref)
    shared = len(set(np.argsort(-eg)[:top]) & set(np.argsort(-ep)[:top]))
    assert shared >= 0.6 * top, (key, shared)


def test_config2_reference_conditioning_probe():
    g = np.load(f"{GOLDEN}/hypergrad_cora_real.npz")
    p = np.load(f"{GOLDEN}/hypergrad_cora_real_probe.npz")
    assert _probe_tol(g, p, "grad0") > 1e-3       # step 0: the reference itself moves by 5e-4
    assert _probe_tol(g, p, "grad1") > GRAD_TOL   # the τ = 5 window: 2.9e-5
    assert np.array_equal(g["inner_losses"], p["inner_losses"])  # losses are not amplified


def test_config2_engine_window_matches_reference_golden():
    """bench.py's default path at its own size: step 0 (1-step window), then
    one captured τ = 5 window replayed from its HIP graph."""
    g = np.load(f"{GOLDEN}/hypergrad_cora_real.npz")
    probe = np.load(f"{GOLDEN}/hypergrad_cora_real_probe.npz")
    seed = int(g["seed"])
    data, inner, outer, gm = _trainers("cora", g, seed)
    eng = engine_from_trainers(inner, outer, tau=5, generator=ldsgnn.rng.default_generator)
    eng.inner_step()
    eng.hyper_step()
    torch.cuda.synchronize()
    losses = [eng.inner_metrics(0)[0]]
    _check_vec(eng.grad, g, "grad0", _probe_tol(g, probe, "grad0"))
    _same_entries_as_probe(eng.grad, g, probe, "grad0")
    _check_vec(eng.theta, g, "theta0", TOL)
    assert gm.probs.grad is eng.grad  # θ.grad holds the hypergradient, as after the reference's backward
    eng.capture_window(5)
    eng.replay(1)
    torch.cuda.synchronize()
    losses += [eng.inner_metrics(t)[0] for t in range(5)]
    assert np.allclose(losses, g["inner_losses"], rtol=TOL, atol=1e-6), (losses, g["inner_losses"])
    _check_vec(eng.grad, g, "grad1", _probe_tol(g, probe, "grad1"))
    _same_entries_as_probe(eng.grad, g, probe, "grad1")
    _check_vec(eng.theta, g, "theta1", TOL)
    p = eng.get_params()
    flat = np.concatenate([p[k].detach().cpu().numpy().ravel() for k in p])
    probe_w = float(np.abs(probe["params_final"] - g["params_final"]).max())
    err = np.abs(flat - g["params_final"])
    assert err.max() <= max(1e-5 * np.abs(g["params_final"]).max(), PROBE_FACTOR * probe_w), (err.max(), probe_w)
    assert (err > 1e-6).sum() <= 10  # only the few ill-conditioned weights move beyond 1e-6


def _vec_err(got, g, key):
    """(max error / max|ref|, L2 relative error) on the golden's picked entries."""
    got = got.detach().double().cpu().numpy()[g["idx"]]
    ref = g[key + "_val"].astype(np.float64)
    err = np.abs(got - ref)
    return float(err.max() / np.abs(ref).max()), float(np.sqrt((err ** 2).sum() / (ref ** 2).sum()))


@pytest.mark.parametrize("dropout", [0.5, 0.0])
def test_config2_wellconditioned_gradients_at_north_star_tolerance(dropout):
    """Kernel error separated from conditioning (golden hypergrad_cora_wellcond,
    made by the reference at config 2's size: real Cora, kNN θ₀): the θ-gradient
    of a hyper step with NO inner step in its window — NLL on the opt mask
    through one sampled outer graph, the weights leaves — has no Adam step
    between θ and the loss to amplify rounding, and the engine holds it (and θ
    after the SGD step) to the north-star 1e-5: every picked entry within
    1e-5 × max|dθ|, ‖dθ‖₂ within 1e-5.  The dropout-free run also checks its
    step-0 window and a whole dropout-free τ = 5 window, whose dθ passes
    through Adam steps (reported in the assertion message; held to 1e-5 where
    the conditioning allows, see test_config2_reference_conditioning_probe)."""
    g = np.load(f"{GOLDEN}/hypergrad_cora_wellcond.npz")
    tag = "" if dropout else "nd_"
    seed = int(g["seed"])
    data, inner, outer, gm = _trainers("cora", g, seed, dropout=dropout)
    eng = engine_from_trainers(inner, outer, tau=5, generator=ldsgnn.rng.default_generator)
    eng.inner_step()
    eng.hyper_step()
    torch.cuda.synchronize()
    assert abs(eng.inner_metrics(0)[0] - float(g[tag + "inner_loss0"])) <= TOL * float(g[tag + "inner_loss0"])
    step0 = _vec_err(eng.grad, g, tag + "grad_step0")
    _check_vec(eng.theta, g, tag + "theta_step0", TOL)
    eng.hyper_step()  # a window with no inner step: the outer graph's path only
    torch.cuda.synchronize()
    outer_err = _vec_err(eng.grad, g, tag + "grad_outer")
    _check_vec(eng.grad, g, tag + "grad_outer", GRAD_TOL)
    _check_vec(eng.theta, g, tag + "theta_outer", TOL)
    if dropout:
        return
    for _ in range(5):
        eng.inner_step()
    eng.hyper_step()
    torch.cuda.synchronize()
    losses = [eng.inner_metrics(t)[0] for t in range(5)]
    assert np.allclose(losses, g["nd_window_losses"], rtol=TOL, atol=1e-6), (losses, g["nd_window_losses"])
    window = _vec_err(eng.grad, g, "nd_grad_window")
    _check_vec(eng.theta, g, "nd_theta_window", TOL)
    diag = {"step0": step0, "outer": outer_err, "window": window}
    print("config2 dropout-free gradient errors (max/max|ref|, L2 rel):", diag)
    assert window[1] <= 1e-5, diag  # the window's dθ as a whole (L2) at the north-star tolerance


def test_config3_citeseer_s16_engine_window_matches_reference_golden():
    """16 replica chains batched in one engine (grid.y = sample), one captured
    τ = 5 window from θ₀: per-replica losses and the mean hypergradient."""
    g = np.load(f"{GOLDEN}/hypergrad_citeseer_s16.npz")
    probe = np.load(f"{GOLDEN}/hypergrad_citeseer_s16_probe.npz")
    seed, S = int(g["seed"]), int(g["samples"])
    data, inner, outer, gm = _trainers("citeseer", g, seed)
    eng = engine_from_trainers(inner, outer, tau=5, generator=ldsgnn.rng.default_generator, samples=S)
    eng.capture_window(5)
    eng.replay(1)
    torch.cuda.synchronize()
    m = eng.metrics.double().cpu().numpy()  # [τ+1, S, 2]: Σ NLL, #correct per replica
    inner_losses = (m[:5, :, 0] * eng.inv_train).T
    outer_losses = m[5, :, 0] * eng.inv_opt
    assert np.allclose(inner_losses, g["inner_losses"], rtol=TOL, atol=1e-6)
    assert np.allclose(outer_losses, g["outer_losses"], rtol=TOL, atol=1e-6)
    _check_vec(eng.grad, g, "grad", _probe_tol(g, probe, "grad"))
    _same_entries_as_probe(eng.grad, g, probe, "grad")
    _check_vec(eng.theta, g, "theta1", TOL)


def test_config3_citeseer_s16_wellconditioned_at_north_star_tolerance():
    """Multi-sample dθ at the north-star 1e-5 (round-5 VERDICT item 6),
    golden hypergrad_citeseer_s16_wellcond (16 reference runners on real
    Citeseer side by side, replica b on the keyed stream of replica b,
    dropout 0, θ set to the mean update after every hyper step): the batched
    S = 16 engine's mean hypergradient of (1) the step-0 window (reported),
    (2) a hyper step with no inner step in its window — every picked entry
    within 1e-5 × max|dθ|, ‖dθ‖₂ within 1e-5 — and (3) a dropout-free τ = 5
    window — ‖dθ‖₂ within 1e-5 (its max entry reported: its Adam steps
    amplify rounding, see test_config2_reference_conditioning_probe).  θ after
    each step, and every replica's losses, within 1e-5."""
    g = np.load(f"{GOLDEN}/hypergrad_citeseer_s16_wellcond.npz")
    seed, S = int(g["seed"]), int(g["samples"])
    data, inner, outer, gm = _trainers("citeseer", g, seed, dropout=0.0)
    eng = engine_from_trainers(inner, outer, tau=5, generator=ldsgnn.rng.default_generator, samples=S)

    def losses_ok(tag, k):
        m = eng.metrics.double().cpu().numpy()
        if k:
            assert np.allclose((m[:k, :, 0] * eng.inv_train).T, g[tag + "_inner_losses"], rtol=TOL, atol=1e-6), tag
        assert np.allclose(m[eng.tau, :, 0] * eng.inv_opt, g[tag + "_outer_losses"], rtol=TOL, atol=1e-6), tag

    errs = {}
    for tag, k in (("step0", 1), ("outer", 0), ("window", 5)):
        for _ in range(k):
            eng.inner_step()
        eng.hyper_step()
        torch.cuda.synchronize()
        losses_ok(tag, k)
        errs[tag] = _vec_err(eng.grad, g, "grad_" + tag)
        _check_vec(eng.theta, g, "theta_" + tag, TOL)
        if tag == "outer":
            _check_vec(eng.grad, g, "grad_outer", GRAD_TOL)
    print("config3 S=16 dropout-free gradient errors (max/max|ref|, L2 rel):", errs)
    assert errs["outer"][0] <= 1e-5 and errs["outer"][1] <= 1e-5, errs
    assert errs["window"][1] <= 1e-5, errs
