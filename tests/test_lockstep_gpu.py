"""Drop-in autograd path vs fused engine, stepped in lockstep on a real
workload (Citeseer, θ pre-training, τ = 20; tools/diag/path_divergence.py).

Both runs start from the same seed: the same θ₀, GCN initialisation and keyed
draws.  For the first few hundred steps they must draw identical graphs
(edge for edge) and keep θ within fp32 rounding of each other — the two
implementations sum in different orders, so they agree to ~1e-7 and then, on
a trajectory of hundreds of Adam steps, drift apart until one Bernoulli draw
crosses its threshold on one path only ("Citeseer at τ = 20").
The bounds here sit before that point for this seed: the first edge flip of
seed 597905256 is at step 422 (profiles/r05_divergence_citeseer.json).
Reference loop: /root/reference/src/trainers/bilevel.py (train: inner step,
hyper step every τ from step 0)."""
import numpy as np
import pytest
import torch

import ldsgnn
from ldsgnn.data.planetoid import load_planetoid_npz
from ldsgnn.fused import engine_from_trainers
from ldsgnn.models.gcn import MetaDenseGCN
from ldsgnn.models.graph import BernoulliGraphModel
from ldsgnn.trainers.bilevel import BilevelProblemRunner
from ldsgnn.trainers.inner import InnerProblemTrainer
from ldsgnn.trainers.outer import OuterProblemTrainer
from ldsgnn.utils.graph import split_mask

SEED, TAU, STEPS = 597905256, 20, 300


def _build(seed, device):
    torch.manual_seed(seed)
    np.random.seed(seed)
    ldsgnn.rng.manual_seed(seed, 0)
    data = load_planetoid_npz("citeseer").to(device)
    data.val_mask, opt_mask = split_mask(data.val_mask, 0.5, shuffle=True)
    opt_mask = opt_mask.to(device)
    data.val_mask = data.val_mask.to(device)
    gcn = MetaDenseGCN(data.num_features, 16, data.num_classes, dropout=0.5).to(device)
    inner = InnerProblemTrainer(gcn, data, lr=0.01, weight_decay=5e-4)
    gm = BernoulliGraphModel(data.dense_adj)
    outer = OuterProblemTrainer(torch.optim.SGD(gm.parameters(), lr=0.1), data, opt_mask, gm, lr_decay=0.99,
                                pretrain=True)
    return data, inner, outer


@pytest.mark.gpu
def test_dropin_and_engine_lockstep_citeseer_tau20(device):
    data, inner_d, outer_d = _build(SEED, device)
    runner = BilevelProblemRunner(inner_d, outer_d, data)
    last = [None]
    orig = outer_d.sample

    def keep():
        last[0] = orig()
        return last[0]
    outer_d.sample = keep
    gen_d = ldsgnn.rng.Generator()
    gen_d.set_state(ldsgnn.rng.default_generator.get_state())
    inner_d.model.generator = gen_d
    outer_d.model.generator = gen_d
    _, inner_e, outer_e = _build(SEED, device)
    eng = engine_from_trainers(inner_e, outer_e, tau=TAU, generator=ldsgnn.rng.default_generator)
    assert torch.equal(outer_d.model.probs.data, eng.theta)
    n = data.num_nodes
    worst_dtheta, worst_loss = 0.0, 0.0
    for step in range(STEPS):
        md = runner.inner_opt_step()
        t = eng.t
        eng.inner_step()
        eng._flush_fill()
        g, ge = last[0], eng.slots[t].g
        nnz = int(ge.row_ptr[0, n].item())
        assert g.nnz() == nnz, f"step {step}: {g.nnz()} vs {nnz} stored entries"
        assert torch.equal(g.row_ptr.int(), ge.row_ptr[0].int()), f"step {step}: row pointers differ"
        assert torch.equal(g.col[:nnz].int(), ge.col[0, :nnz].int()), f"step {step}: edges differ"
        le = eng.inner_metrics(t)[0]
        worst_loss = max(worst_loss, abs(float(md.loss) - le) / abs(le))
        if step % TAU == 0:
            runner.hyper_opt_step(step)
            eng.hyper_step()
            worst_dtheta = max(worst_dtheta, float((outer_d.model.probs.data - eng.theta).abs().max()))
    # fp32 rounding of two summation orders, nothing more
    assert worst_dtheta <= 1e-6, worst_dtheta
    assert worst_loss <= 1e-5, worst_loss
