"""The CPU oracle (oracle/lds_oracle.py) pinned against the reference-made
goldens of the BASELINE workloads (tests/golden/make_golden.py):

  gcn_fixed_cora          config 1: FixedGcnTraining vs the reference's
                          src/scripts/gcn.py loop on real Cora
  hypergrad_cora_real     config 2: LdsProblem vs the reference's step-0 hyper
                          step and τ = 5 window on real Cora with the kNN θ₀
  hypergrad_citeseer_s16  config 3: replica 0's chain vs the reference's
                          replica-0 runner on real Citeseer (the golden's other
                          15 replicas are exercised on the GPU only)
"""
import numpy as np
import pytest
import torch

from ldsgnn.data.workloads import load_workload
from oracle import lds_oracle as O
from tests.conftest import GOLDEN


def _gold(name):
    return np.load(f"{GOLDEN}/{name}.npz")


def test_oracle_fixed_gcn_matches_reference_golden():
    g = _gold("gcn_fixed_cora")
    seed = int(g["seed"])
    data = load_workload("cora-given")
    torch.manual_seed(seed)
    params = O.reference_construction_params(data.num_features, 16, data.num_classes)
    p0 = np.concatenate([p.numpy().ravel() for p in params.values()])
    assert np.array_equal(p0, g["params0"])
    run = O.FixedGcnTraining(data.x, data.y, data.dense_adj, data.train_mask, data.val_mask, data.test_mask,
                             rnd=O.Randomness(seed), params=params)
    epochs = 25
    for e in range(epochs):
        loss, acc, m = run.epoch()
        want = g["rows"][e]
        assert np.allclose([loss, m["val.loss"], m["test.loss"]], want[[0, 2, 4]], rtol=1e-5, atol=1e-6), e
        assert np.allclose([acc, m["val.accuracy"], m["test.accuracy"]], want[[1, 3, 5]], atol=1e-6), e


def _problem(workload, g, replica=0):
    seed = int(g["seed"])
    data = load_workload(workload)
    torch.manual_seed(seed)
    params = O.reference_construction_params(data.num_features, 16, data.num_classes)
    opt = torch.from_numpy(g["opt_mask"])
    return O.LdsProblem(data.x, data.y, data.train_mask, torch.from_numpy(g["val_mask"]), data.test_mask, opt,
                        O.get_triu_values(data.dense_adj), dropout_p=0.5, outer_lr=0.1, lr_decay=0.99,
                        rnd=O.Randomness(seed, replica), params=params)


def _close_vec(got, g, key, rtol):
    got = got.detach().double().numpy()
    ref = g[key + "_val"].astype(np.float64)
    scale = np.abs(ref).max()
    assert np.all(np.abs(got[g["idx"]] - ref) <= rtol * np.abs(ref) + 1e-6 * scale), key
    assert np.isclose(np.sqrt((got ** 2).sum()), float(g[key + "_l2"]), rtol=1e-5), key


@pytest.mark.slow
def test_oracle_cora_knn_windows_match_reference_golden():
    g = _gold("hypergrad_cora_real")
    prob = _problem("cora", g)
    losses, grads, thetas = [], [], []
    for step in range(6):
        losses.append(prob.inner_step(prob.sample())[0])
        if step % 5 == 0:
            grads.append(prob.hyper_step()[2])
            thetas.append(prob.theta.detach().clone())
    assert np.allclose(losses, g["inner_losses"], rtol=1e-5, atol=1e-6)
    for h in range(2):
        _close_vec(grads[h], g, f"grad{h}", 1e-4)
        _close_vec(thetas[h], g, f"theta{h}", 1e-5)


@pytest.mark.slow
def test_oracle_citeseer_replica0_matches_reference_golden():
    g = _gold("hypergrad_citeseer_s16")
    prob = _problem("citeseer", g, replica=0)
    losses = [prob.inner_step(prob.sample())[0] for _ in range(5)]
    outer = prob.hyper_grad()[0]
    assert np.allclose(losses, g["inner_losses"][0], rtol=1e-5, atol=1e-6)
    assert np.isclose(outer, g["outer_losses"][0], rtol=1e-5, atol=1e-6)
