"""Test infrastructure: run the product (ldsgnn on cuda:0) and the CPU oracle
on the same seeded synthetic LDS problem and report the largest differences.
Used by tests/ and __graft_entry__.smoke()."""
from __future__ import annotations

from collections import OrderedDict

import numpy as np
import torch

from oracle import lds_oracle as O


def synthetic_problem(n: int, f_in: int, classes: int, seed: int, p_edge: float = 0.05):
    g = torch.Generator().manual_seed(seed)
    x = torch.rand(n, f_in, generator=g) * (torch.rand(n, f_in, generator=g) < 0.3)
    x = x / x.sum(1, keepdim=True).clamp(min=1e-12)  # NormalizeFeatures
    y = torch.randint(0, classes, (n,), generator=g)
    perm = torch.randperm(n, generator=g)
    ntr, nva = max(2, n // 5), max(2, (3 * n) // 10)
    masks = []
    for idx in (perm[:ntr], perm[ntr:ntr + nva // 2], perm[ntr + nva // 2:ntr + nva], perm[ntr + nva:]):
        m = torch.zeros(n, dtype=torch.bool)
        m[idx] = True
        masks.append(m)
    train, val, opt, test = masks
    a = (torch.rand(n, n, generator=g) < p_edge).float().triu(1)
    adj = a + a.t()
    return dict(x=x, y=y, train=train, val=val, opt=opt, test=test, adj=adj)


def build_product(prob, hidden=16, dropout=0.5, gcn_lr=0.01, gcn_wd=5e-4, outer_lr=0.1,
                  lr_decay=0.99, seed=0, device="cuda"):
    import ldsgnn
    from ldsgnn.models.gcn import MetaDenseGCN
    from ldsgnn.models.graph import BernoulliGraphModel
    from ldsgnn.trainers.bilevel import BilevelProblemRunner
    from ldsgnn.trainers.inner import InnerProblemTrainer
    from ldsgnn.trainers.outer import OuterProblemTrainer
    from ldsgnn.utils.graph import DenseData

    data = DenseData(x=prob["x"], y=prob["y"], dense_adj=prob["adj"], train_mask=prob["train"],
                     val_mask=prob["val"], test_mask=prob["test"],
                     num_classes=int(prob["y"].max()) + 1).to(device)
    ldsgnn.rng.manual_seed(seed, 0)
    torch.manual_seed(seed)
    gcn = MetaDenseGCN(data.num_features, hidden, data.num_classes, dropout=dropout).to(device)
    inner = InnerProblemTrainer(gcn, data, lr=gcn_lr, weight_decay=gcn_wd)
    gm = BernoulliGraphModel(data.dense_adj)
    opt = torch.optim.SGD(gm.parameters(), lr=outer_lr)
    outer = OuterProblemTrainer(opt, data, prob["opt"].to(device), gm, lr_decay=lr_decay)
    runner = BilevelProblemRunner(inner, outer, data)
    return runner


def build_product_embedding(prob, hidden=16, dropout=0.5, gcn_lr=0.01, gcn_wd=5e-4, outer_lr=0.5,
                            lr_decay=0.99, seed=0, embedding_dim=8, init_bounds=0.3, device="cuda"):
    """build_product with the embedding graph model (P = σ(E·Eᵀ), SGD on E,
    src/models/graph.py:81-112, src/models/factory.py embeddings_optimizer)."""
    import ldsgnn
    from ldsgnn.models.gcn import MetaDenseGCN
    from ldsgnn.models.graph import PairwiseEmbeddingSampler
    from ldsgnn.trainers.bilevel import BilevelProblemRunner
    from ldsgnn.trainers.inner import InnerProblemTrainer
    from ldsgnn.trainers.outer import OuterProblemTrainer
    from ldsgnn.utils.graph import DenseData

    data = DenseData(x=prob["x"], y=prob["y"], dense_adj=prob["adj"], train_mask=prob["train"],
                     val_mask=prob["val"], test_mask=prob["test"],
                     num_classes=int(prob["y"].max()) + 1).to(device)
    ldsgnn.rng.manual_seed(seed, 0)
    torch.manual_seed(seed)
    gcn = MetaDenseGCN(data.num_features, hidden, data.num_classes, dropout=dropout).to(device)
    inner = InnerProblemTrainer(gcn, data, lr=gcn_lr, weight_decay=gcn_wd)
    gm = PairwiseEmbeddingSampler(data.num_nodes, embedding_dim, init_bounds=init_bounds).to(device)
    opt = torch.optim.SGD(gm.parameters(), lr=outer_lr)
    outer = OuterProblemTrainer(opt, data, prob["opt"].to(device), gm, lr_decay=lr_decay)
    return BilevelProblemRunner(inner, outer, data)


def build_product_gae(prob, hidden=16, dropout=0.5, gcn_lr=0.01, gcn_wd=5e-4, lr_decay=0.99, seed=0,
                      embedding_dim=8, device="cuda", proposal_dropout=0.0):
    """build_product with the GAE graph model (proposal GCN with dropout
    `proposal_dropout`, P = clamp(σ(a·E·Eᵀ + b), 0, 1); Adam on the GCN,
    SGD-rate on a, b as src/models/factory.py:51-57 groups them)."""
    import ldsgnn
    from ldsgnn.models.gcn import MetaDenseGCN
    from ldsgnn.models.graph import GraphProposalNetwork
    from ldsgnn.trainers.bilevel import BilevelProblemRunner
    from ldsgnn.trainers.inner import InnerProblemTrainer
    from ldsgnn.trainers.outer import OuterProblemTrainer
    from ldsgnn.utils.graph import DenseData

    data = DenseData(x=prob["x"], y=prob["y"], dense_adj=prob["adj"], train_mask=prob["train"],
                     val_mask=prob["val"], test_mask=prob["test"],
                     num_classes=int(prob["y"].max()) + 1).to(device)
    ldsgnn.rng.manual_seed(seed, 0)
    torch.manual_seed(seed)
    gcn = MetaDenseGCN(data.num_features, hidden, data.num_classes, dropout=dropout).to(device)
    inner = InnerProblemTrainer(gcn, data, lr=gcn_lr, weight_decay=gcn_wd)
    gm = GraphProposalNetwork(data.x, data.dense_adj, dropout=proposal_dropout, embedding_dim=embedding_dim).to(device)
    opt = torch.optim.Adam([{"params": gm.gcn.parameters(), "weight_decay": 5e-4, "lr": 0.01},
                            {"params": [gm.probs_factor, gm.probs_bias], "lr": 0.01}])
    outer = OuterProblemTrainer(opt, data, prob["opt"].to(device), gm, lr_decay=lr_decay)
    return BilevelProblemRunner(inner, outer, data)


def build_oracle(prob, runner, hidden=16, dropout=0.5, gcn_lr=0.01, gcn_wd=5e-4, outer_lr=0.1,
                 lr_decay=0.99, seed=0):
    params = OrderedDict((k, v.detach().cpu()) for k, v in runner.inner_trainer.model_params.items())
    theta = O.get_triu_values(prob["adj"])
    return O.LdsProblem(prob["x"], prob["y"], prob["train"], prob["val"], prob["test"], prob["opt"],
                        theta, hidden=hidden, dropout_p=dropout, gcn_lr=gcn_lr, gcn_wd=gcn_wd,
                        outer_lr=outer_lr, lr_decay=lr_decay, rnd=O.Randomness(seed, 0), params=params)


def run_product_and_oracle(n=96, f_in=24, classes=4, steps=6, tau=5, dropout=0.5, seed=0,
                           hidden=16, p_edge=0.05):
    prob = synthetic_problem(n, f_in, classes, seed, p_edge)
    runner = build_product(prob, hidden=hidden, dropout=dropout, seed=seed)
    oracle = build_oracle(prob, runner, hidden=hidden, dropout=dropout, seed=seed)
    p_losses, o_losses, p_outer, o_outer = [], [], [], []
    for step in range(steps):
        p_losses.append(runner.inner_opt_step().loss)
        o_losses.append(oracle.inner_step(oracle.sample())[0])
        if tau == 0 or step % tau == 0:
            p_outer.append(runner.hyper_opt_step(step).loss)
            o_outer.append(oracle.hyper_step()[0])
    theta_p = runner.outer_trainer.model.probs.detach().cpu()
    theta_o = oracle.theta.detach()
    perr = max(float((a.detach().cpu() - b.detach()).abs().max())
               for a, b in zip(runner.inner_trainer.model_params.values(), oracle.params.values()))
    return dict(
        max_theta_err=float((theta_p - theta_o).abs().max()),
        max_param_err=perr,
        max_loss_err=float(np.max(np.abs(np.array(p_losses + p_outer) - np.array(o_losses + o_outer)))),
        theta_changed=float((theta_o - O.get_triu_values(prob["adj"])).abs().max()),
        losses=p_losses, outer=p_outer,
    )


def run_engine_and_oracle(n=96, f_in=24, classes=4, steps=6, tau=5, dropout=0.5, seed=0, p_edge=0.05,
                          hidden=16, theta_uniform=None, **engine_kwargs):
    """Fused engine (ldsgnn.engine) vs the oracle on the same problem: per-step
    inner losses, final GCN params, every θ-gradient and the final θ."""
    import ldsgnn
    from ldsgnn.engine import LdsEngine
    from ldsgnn.models.gcn import MetaDenseGCN
    prob = synthetic_problem(n, f_in, classes, seed, p_edge)
    torch.manual_seed(seed)
    gcn = MetaDenseGCN(f_in, hidden, classes, dropout=dropout)
    params = OrderedDict((k, v.detach()) for k, v in gcn.named_parameters())
    dev = "cuda"
    theta0 = O.get_triu_values(prob["adj"])
    if theta_uniform is not None:  # dense θ ~ U(0, theta_uniform) (config 5's kind of graph)
        theta0 = torch.rand(theta0.numel(), generator=torch.Generator().manual_seed(seed + 1)) * theta_uniform
    theta = theta0.clone().to(dev).contiguous()
    eng = LdsEngine(prob["x"].to(dev), prob["y"].to(dev), prob["train"].to(dev), prob["opt"].to(dev), theta,
                    classes, dropout=dropout, gcn_lr=0.01, gcn_wd=5e-4, outer_lr=0.1, lr_decay=0.99, tau=tau,
                    generator=ldsgnn.rng.Generator(seed, 0), params=OrderedDict((k, v.to(dev)) for k, v in params.items()),
                    **engine_kwargs)
    oracle = O.LdsProblem(prob["x"], prob["y"], prob["train"], prob["val"], prob["test"], prob["opt"],
                          theta0.clone(), hidden=hidden, dropout_p=dropout, gcn_lr=0.01,
                          gcn_wd=5e-4, outer_lr=0.1, lr_decay=0.99, rnd=O.Randomness(seed, 0), params=params)
    e_losses, o_losses, gerr, grel = [], [], [], []
    for step in range(steps):
        t = eng.t
        eng.inner_step()
        e_losses.append(eng.inner_metrics(t)[0])
        o_losses.append(oracle.inner_step(oracle.sample())[0])
        if tau == 0 or step % tau == 0:
            eng.hyper_step()
            og = oracle.hyper_step()[2]
            eg = eng.grad.detach().cpu()
            gerr.append(float((eg - og).abs().max()))
            grel.append(float((eg - og).abs().max() / og.abs().max().clamp(min=1e-30)))
    eparams = eng.get_params()
    perr = max(float((eparams[k].cpu() - oracle.params[k].detach()).abs().max()) for k in eparams)
    return dict(max_loss_err=float(np.max(np.abs(np.array(e_losses) - np.array(o_losses)))),
                max_param_err=perr, max_grad_err=max(gerr) if gerr else 0.0,
                max_grad_rel=max(grel) if grel else 0.0,
                max_theta_err=float((eng.theta.cpu() - oracle.theta.detach()).abs().max()),
                theta_changed=float((oracle.theta.detach() - theta0).abs().max()),
                engine=eng, oracle=oracle)


def run_engine_samples_and_oracle(samples=3, n=96, f_in=24, classes=4, steps=6, tau=5, dropout=0.5, seed=0,
                                  p_edge=0.05, hidden=16, replica0=0):
    """Batched engine (S replica samples in one launch set) vs S oracle
    replicas (Randomness replica replica0 + b) sharing θ and updated by the
    mean hypergradient (oracle.replica_hyper_step)."""
    import ldsgnn
    from ldsgnn.engine import LdsEngine
    from ldsgnn.models.gcn import MetaDenseGCN
    prob = synthetic_problem(n, f_in, classes, seed, p_edge)
    torch.manual_seed(seed)
    gcn = MetaDenseGCN(f_in, hidden, classes, dropout=dropout)
    params = OrderedDict((k, v.detach()) for k, v in gcn.named_parameters())
    dev = "cuda"
    theta = O.get_triu_values(prob["adj"]).to(dev).contiguous()
    eng = LdsEngine(prob["x"].to(dev), prob["y"].to(dev), prob["train"].to(dev), prob["opt"].to(dev), theta,
                    classes, dropout=dropout, gcn_lr=0.01, gcn_wd=5e-4, outer_lr=0.1, lr_decay=0.99, tau=tau,
                    generator=ldsgnn.rng.Generator(seed, replica0),
                    params=OrderedDict((k, v.to(dev)) for k, v in params.items()), samples=samples)
    oracles = [O.LdsProblem(prob["x"], prob["y"], prob["train"], prob["val"], prob["test"], prob["opt"],
                            O.get_triu_values(prob["adj"]), hidden=hidden, dropout_p=dropout, gcn_lr=0.01,
                            gcn_wd=5e-4, outer_lr=0.1, lr_decay=0.99, rnd=O.Randomness(seed, replica0 + b),
                            params=params) for b in range(samples)]
    lerr, grel = [], []
    for step in range(steps):
        t = eng.t
        eng.inner_step()
        e_rows = eng.metrics[t].cpu().numpy()  # [S, 2] Σ loss, #correct
        for b, orc in enumerate(oracles):
            ol = orc.inner_step(orc.sample())[0]
            lerr.append(abs(float(e_rows[b, 0]) * eng.inv_train - ol))
        if tau == 0 or step % tau == 0:
            eng.hyper_step()
            outs, og = O.replica_hyper_step(oracles)
            e_rows = eng.metrics[eng.tau].cpu().numpy()
            for b, (ol, _) in enumerate(outs):
                lerr.append(abs(float(e_rows[b, 0]) * eng.inv_opt - ol))
            eg = eng.grad.detach().cpu()
            grel.append(float((eg - og).abs().max() / og.abs().max().clamp(min=1e-30)))
    perr = 0.0
    for b, orc in enumerate(oracles):
        ep = eng.get_params(b)
        perr = max(perr, max(float((ep[k].cpu() - orc.params[k].detach()).abs().max()) for k in ep))
    terr = max(float((eng.theta.cpu() - orc.theta.detach()).abs().max()) for orc in oracles)
    return dict(max_loss_err=float(max(lerr)) if lerr else 0.0, max_param_err=perr, max_grad_rel=max(grel) if grel else 0.0,
                max_theta_err=terr,
                theta_changed=float((oracles[0].theta.detach() - O.get_triu_values(prob["adj"])).abs().max()),
                engine=eng, oracles=oracles)
