"""End-to-end parity of the drop-in trainers (HIP path) with the CPU oracle:
inner losses, GCN parameters after differentiable-Adam steps, and θ after the
truncated-hypergradient SGD steps.  fp32 tolerance 1e-5 (north_star)."""
import pytest

from tests.parity_harness import run_product_and_oracle

pytestmark = pytest.mark.gpu

TOL = 1e-5


@pytest.mark.parametrize("dropout", [0.0, 0.5])
@pytest.mark.parametrize("tau", [1, 5])
def test_bilevel_steps_match_oracle(dropout, tau):
    res = run_product_and_oracle(n=96, f_in=24, classes=4, steps=11, tau=tau, dropout=dropout, seed=3)
    assert res["theta_changed"] > 0  # the hypergradient did move θ
    assert res["max_loss_err"] < TOL, res
    assert res["max_param_err"] < TOL, res
    assert res["max_theta_err"] < TOL, res


def test_bilevel_dense_theta_graph():
    """θ fractional and dense-ish (p_edge 0.3): long CSR rows, many slots."""
    res = run_product_and_oracle(n=150, f_in=40, classes=5, steps=6, tau=5, dropout=0.5, seed=5,
                                 p_edge=0.3)
    assert res["max_loss_err"] < TOL, res
    assert res["max_param_err"] < TOL, res
    assert res["max_theta_err"] < TOL, res
