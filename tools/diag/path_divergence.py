"""Where the drop-in autograd path and the fused engine part ways on one
seed of the accuracy runs (tools/accuracy_run.py: real Planetoid split, θ
pre-training, τ given): both are built from the same seed (same θ₀, same GCN
initialisation, same keyed draws) and stepped in lockstep — inner steps,
hyper steps every τ — with no early stopping.  Per step: the sampled graph's
stored entries on each path (the first step whose draws differ), and after
every hyper step max|Δθ| and the inner-loss difference.  One JSON line.

  python tools/diag/path_divergence.py --dataset citeseer --seed 597905257 --tau 20 --steps 3000
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lds-gnn_amd"), os.path.join(ROOT, "tools")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import ldsgnn  # noqa: E402
from ldsgnn.data.planetoid import load_planetoid_npz  # noqa: E402
from ldsgnn.fused import engine_from_trainers  # noqa: E402
from ldsgnn.models.gcn import MetaDenseGCN  # noqa: E402
from ldsgnn.models.graph import BernoulliGraphModel  # noqa: E402
from ldsgnn.trainers.bilevel import BilevelProblemRunner  # noqa: E402
from ldsgnn.trainers.inner import InnerProblemTrainer  # noqa: E402
from ldsgnn.trainers.outer import OuterProblemTrainer  # noqa: E402
from ldsgnn.utils.graph import split_mask  # noqa: E402


def build(dataset, seed, device):
    torch.manual_seed(seed)
    np.random.seed(seed)
    ldsgnn.rng.manual_seed(seed, 0)
    data = load_planetoid_npz(dataset).to(device)
    data.val_mask, opt_mask = split_mask(data.val_mask, 0.5, shuffle=True)
    opt_mask = opt_mask.to(device)
    data.val_mask = data.val_mask.to(device)
    gcn = MetaDenseGCN(data.num_features, 16, data.num_classes, dropout=0.5).to(device)
    inner = InnerProblemTrainer(gcn, data, lr=0.01, weight_decay=5e-4)
    gm = BernoulliGraphModel(data.dense_adj)
    outer = OuterProblemTrainer(torch.optim.SGD(gm.parameters(), lr=0.1), data, opt_mask, gm, lr_decay=0.99,
                                pretrain=True)
    return data, inner, outer


_last_graph = [None]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dataset", default="citeseer")
    ap.add_argument("--seed", type=int, default=597905257)
    ap.add_argument("--tau", type=int, default=20)
    ap.add_argument("--steps", type=int, default=3000)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    data, inner_d, outer_d = build(args.dataset, args.seed, dev)
    runner = BilevelProblemRunner(inner_d, outer_d, data)
    orig_sample = outer_d.sample

    def sample_and_keep():
        g = orig_sample()
        _last_graph[0] = g
        return g
    outer_d.sample = sample_and_keep
    # the drop-in path keeps a private copy of the generator state after its
    # build; the second build reseeds the default generator for the engine
    gen_d = ldsgnn.rng.Generator()
    gen_d.set_state(ldsgnn.rng.default_generator.get_state())
    inner_d.model.generator = gen_d
    outer_d.model.generator = gen_d
    _, inner_e, outer_e = build(args.dataset, args.seed, dev)
    eng = engine_from_trainers(inner_e, outer_e, tau=args.tau, generator=ldsgnn.rng.default_generator)
    out = {"dataset": args.dataset, "seed": args.seed, "tau": args.tau, "steps": args.steps,
           "theta0_equal": bool(torch.equal(outer_d.model.probs.data, eng.theta))}
    hyper, loss_diff, graph_diffs = [], [], []
    n = data.num_nodes
    for step in range(args.steps):
        md = runner.inner_opt_step()
        t = eng.t
        eng.inner_step()
        eng._flush_fill()
        if len(graph_diffs) < 8:
            ge = eng.slots[t].g
            nnz_e = int(ge.row_ptr[0, n].item())
            g = _last_graph[0]
            if g is not None:
                same = g.nnz() == nnz_e and torch.equal(g.row_ptr.int(), ge.row_ptr[0].int()) and \
                    torch.equal(g.col[:nnz_e].int(), ge.col[0, :nnz_e].int())
                if not same:
                    graph_diffs.append({"step": step, "nnz_dropin": g.nnz(), "nnz_engine": nnz_e})
        le = eng.inner_metrics(t)[0]
        loss_diff.append(abs(float(md.loss) - le) / max(abs(le), 1e-30))
        if step % args.tau == 0:
            mo = runner.hyper_opt_step(step)
            eng.hyper_step()
            lo = eng.outer_metrics()[0]
            dth = float((outer_d.model.probs.data - eng.theta).abs().max())
            hyper.append({"step": step, "max_dtheta": dth, "inner_loss_rel_diff": loss_diff[-1],
                          "outer_loss_rel_diff": abs(float(mo.loss) - lo) / max(abs(lo), 1e-30)})
        if step % 200 == 0:
            print(f"step {step}", file=sys.stderr, flush=True)
    out["graph_differences"] = graph_diffs
    for thr in (1e-6, 1e-4, 1e-2):
        out[f"first_step_inner_loss_rel_diff_above_{thr:g}"] = next(
            (i for i, d in enumerate(loss_diff) if d > thr), None)
    for thr in (1e-6, 1e-5, 1e-4, 1e-3, 1e-2):
        hit = next((h["step"] for h in hyper if h["max_dtheta"] > thr), None)
        out[f"first_hyper_step_dtheta_above_{thr:g}"] = hit
    if graph_diffs:
        s0 = graph_diffs[0]["step"]
        out["hyper_around_first_graph_difference"] = [h for h in hyper if s0 - 3 * args.tau <= h["step"] <= s0 + 3 * args.tau]
    out["hyper"] = hyper[:: max(1, len(hyper) // 40)]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
