"""The fused engine (hand-derived reverse pass, csrc/engine.hip) against the
CPU oracle and the reference goldens; HIP-graph replay against eager."""
import numpy as np
import pytest
import torch

from tests.parity_harness import run_engine_and_oracle

pytestmark = pytest.mark.gpu
TOL = 1e-5


@pytest.mark.parametrize("dropout", [0.0, 0.5])
@pytest.mark.parametrize("tau", [1, 5])
def test_engine_matches_oracle(dropout, tau):
    res = run_engine_and_oracle(n=96, f_in=24, classes=4, steps=11, tau=tau, dropout=dropout, seed=3)
    assert res["theta_changed"] > 0
    assert res["max_loss_err"] < TOL, res
    assert res["max_param_err"] < TOL, res
    assert res["max_grad_rel"] < 1e-4, res
    assert res["max_theta_err"] < TOL, res


def test_engine_dense_theta_seven_classes():
    res = run_engine_and_oracle(n=150, f_in=40, classes=7, steps=6, tau=5, dropout=0.5, seed=5, p_edge=0.3)
    assert res["max_loss_err"] < TOL, res
    assert res["max_param_err"] < TOL, res
    assert res["max_grad_rel"] < 1e-4, res
    assert res["max_theta_err"] < TOL, res


def test_graph_replay_equals_eager():
    """A captured τ-window replays exactly like eager windows (same RNG draws,
    Adam steps, lr decay): bitwise-identical θ and weights."""
    a = run_engine_and_oracle(n=130, f_in=30, classes=5, steps=1, tau=5, dropout=0.5, seed=9)["engine"]
    b = run_engine_and_oracle(n=130, f_in=30, classes=5, steps=1, tau=5, dropout=0.5, seed=9)["engine"]
    a.capture_window(5)
    a.replay(3)
    for _ in range(3):
        b.run_window(5)
    torch.cuda.synchronize()
    assert torch.equal(a.theta, b.theta)
    for k, v in a.get_params().items():
        assert torch.equal(v, b.get_params()[k]), k
    assert a.scalars_host() == b.scalars_host()


def test_batched_window_sampling_equals_stepwise():
    """run_window draws the window's graphs in one batched launch set: same
    draws (counters), same results as sampling step by step."""
    a = run_engine_and_oracle(n=140, f_in=30, classes=6, steps=1, tau=5, dropout=0.5, seed=21)["engine"]
    b = run_engine_and_oracle(n=140, f_in=30, classes=6, steps=1, tau=5, dropout=0.5, seed=21)["engine"]
    for _ in range(2):
        a.run_window(5)  # batched sampling
        for _ in range(5):  # step by step
            b.inner_step()
        b.hyper_step()
    torch.cuda.synchronize()
    assert torch.equal(a.theta, b.theta)
    for k, v in a.get_params().items():
        assert torch.equal(v, b.get_params()[k]), k


def test_split_graph_replay_with_reducer_equals_eager():
    """N>1 capture: the window is split at the θ-grad exchange (graph A, the
    reducer run eagerly, graph B).  Replays must equal eager windows that call
    the same reducer, and the reducer must really act between the graphs."""
    calls = []

    def halve(grad):  # stands in for all_reduce(SUM)/world
        calls.append(1)
        grad.mul_(0.5)

    a = run_engine_and_oracle(n=130, f_in=30, classes=5, steps=1, tau=5, dropout=0.5, seed=9)["engine"]
    b = run_engine_and_oracle(n=130, f_in=30, classes=5, steps=1, tau=5, dropout=0.5, seed=9)["engine"]
    c = run_engine_and_oracle(n=130, f_in=30, classes=5, steps=1, tau=5, dropout=0.5, seed=9)["engine"]
    a.capture_window(5, grad_reducer=halve)
    calls.clear()
    a.replay(3)
    assert len(calls) == 3
    for _ in range(3):
        b.run_window(5, grad_reducer=halve)
        c.run_window(5)
    torch.cuda.synchronize()
    assert torch.equal(a.theta, b.theta)
    assert torch.equal(a.grad, b.grad)
    assert not torch.equal(a.theta, c.theta)  # the halved gradient moved θ differently
    for k, v in a.get_params().items():
        assert torch.equal(v, b.get_params()[k]), k
    assert a.scalars_host() == b.scalars_host()
