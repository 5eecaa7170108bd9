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
    gen_d = ldsgnn.rng.default_generator
    _, inner_e, outer_e = build(args.dataset, args.seed, dev)
    eng = engine_from_trainers(inner_e, outer_e, tau=args.tau, generator=ldsgnn.rng.default_generator)
    # the two builds each reseeded the default generator; the drop-in trainers
    # keep theirs through the model's generator attribute where they have one
    out = {"dataset": args.dataset, "seed": args.seed, "tau": args.tau, "steps": args.steps,
           "theta0_equal": bool(torch.equal(outer_d.model.probs.data, eng.theta))}
    first_draw_diff, hyper = None, []
    n = data.num_nodes
    for step in range(args.steps):
        runner.outer_trainer.train()
        g = runner.outer_trainer.sample()
        md = runner.inner_trainer.train_step(g)
        t = eng.t
        eng.inner_step()
        nnz_e = int(eng.slots[t].g.row_ptr[0, n].item())
        if first_draw_diff is None and g.nnz() != nnz_e:
            first_draw_diff = {"step": step, "nnz_dropin": g.nnz(), "nnz_engine": nnz_e}
        if step % args.tau == 0:
            runner.hyper_opt_step(step)
            eng.hyper_step()
            le = eng.inner_metrics(t)[0]
            dth = float((outer_d.model.probs.data - eng.theta).abs().max())
            hyper.append({"step": step, "max_dtheta": dth, "inner_loss_diff": abs(float(md.loss) - le)})
    out["first_draw_difference"] = first_draw_diff
    for thr in (1e-6, 1e-5, 1e-4, 1e-3, 1e-2):
        hit = next((h["step"] for h in hyper if h["max_dtheta"] > thr), None)
        out[f"first_hyper_step_dtheta_above_{thr:g}"] = hit
    out["hyper"] = hyper[:: max(1, len(hyper) // 40)]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
