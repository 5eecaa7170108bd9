"""Accuracy of the MI355X path on the real Planetoid split — the reference's
final LDS configuration (configs/seml/final/lds.yaml: τ = 5, patience 20,
16 evaluation samples, GCN lr 0.01 / wd 5e-4 / dropout 0.5 / hidden 16, θ lr
0.1 with decay 0.99, θ pre-training on, θ₀ = the given graph,
shuffle_splits False) and the GCN baseline (src/scripts/gcn.py defaults: Adam
lr 0.01, wd 5e-4 on layer_in, 200 epochs, patience 10), through the drop-in
API (src/scripts/bilevel.py:73-111, src/scripts/gcn.py:50-100).  Published:
report.pdf p.8 Table 3 — LDS 84.2 ± 0.5 (Cora), 74.0 ± 0.5 (Citeseer); GCN
81.2 ± 0.4 / 70.8 ± 0.5.  One JSON line per run, then a summary line.

  python tools/accuracy_run.py --dataset cora --seeds 5 [--model lds|gcn]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "lds-gnn_amd")):
    sys.path.insert(0, p)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import ldsgnn  # noqa: E402
from ldsgnn.data.planetoid import load_planetoid_npz  # noqa: E402
from ldsgnn.models.gcn import MetaDenseGCN  # noqa: E402
from ldsgnn.models.graph import BernoulliGraphModel  # noqa: E402
from ldsgnn.trainers.bilevel import BilevelProblemRunner  # noqa: E402
from ldsgnn.trainers.inner import InnerProblemTrainer  # noqa: E402
from ldsgnn.trainers.outer import OuterProblemTrainer  # noqa: E402
from ldsgnn.utils.early_stopping import EarlyStopping  # noqa: E402
from ldsgnn.utils.evaluation import evaluate  # noqa: E402
from ldsgnn.utils.graph import split_mask  # noqa: E402

PUBLISHED = {("lds", "cora"): (84.2, 0.5), ("lds", "citeseer"): (74.0, 0.5),
             ("gcn", "cora"): (81.2, 0.4), ("gcn", "citeseer"): (70.8, 0.5)}


def run_lds(dataset, seed, device, pretrain=True, tau=5, fused=False):
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
                                pretrain=pretrain)
    steps = {"inner": 0}
    if fused:  # the fused engine drives the whole loop (ldsgnn.fused.FusedBilevelRunner)
        from ldsgnn.fused import FusedBilevelRunner
        runner = FusedBilevelRunner(inner, outer, data, n_samples_empirical_mean=16)
    else:
        runner = BilevelProblemRunner(inner, outer, data, n_samples_empirical_mean=16)
        orig = runner.inner_opt_step

        def counted():
            steps["inner"] += 1
            return orig()
        runner.inner_opt_step = counted
    def progress(name, value, step=None):  # outer-epoch heartbeat (keeps long runs visibly alive)
        if fused and name == "loss.train":
            steps["inner"] += 1
        if name == "loss.val.empirical":
            print(f"  seed {seed} step {steps['inner']} {name}={value:.4f}", file=sys.stderr, flush=True)
    runner.train(patience=20, hyper_gradient_interval=tau, sacred_runner=progress)
    res = runner.evaluate()
    res["inner_steps"] = steps["inner"]
    res["pretrain"] = outer.pretrain_results
    return res


def run_gcn(dataset, seed, device, epochs=200, patience=10):
    torch.manual_seed(seed)
    np.random.seed(seed)
    ldsgnn.rng.manual_seed(seed, 0)
    data = load_planetoid_npz(dataset).to(device)
    from ldsgnn.ops import csr_graph_from_dense
    data.graph = csr_graph_from_dense(data.dense_adj)
    gcn = MetaDenseGCN(data.num_features, 16, data.num_classes, dropout=0.5).to(device)
    opt = torch.optim.Adam([{"params": gcn.layer_in.parameters(), "weight_decay": 5e-4},
                            {"params": gcn.layer_out.parameters()}], lr=0.01)
    stopper = EarlyStopping(patience)
    for _ in range(epochs):
        opt.zero_grad()
        gcn.train()
        out = gcn(data.x, data.graph)
        loss = F.nll_loss(out[data.train_mask], data.y[data.train_mask])
        loss.backward()
        opt.step()
        m = evaluate(gcn, data)
        stopper.update(m["val.loss"], model=gcn)
        if stopper.abort:
            break
    gcn.load_state_dict(stopper.best_model_state_dict())
    m = evaluate(gcn, data)
    return {"acc.test.final": m["test.accuracy"], "acc.val.final": m["val.accuracy"],
            "loss.test.final": m["test.loss"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dataset", default="cora")
    ap.add_argument("--model", default="lds", choices=["lds", "gcn"])
    ap.add_argument("--seeds", type=int, default=5)
    ap.add_argument("--seed0", type=int, default=597905255 % (2 ** 31))
    ap.add_argument("--no-pretrain", action="store_true")
    ap.add_argument("--tau", type=int, default=5)
    ap.add_argument("--fused", action="store_true", help="drive the loop with the fused engine")
    args = ap.parse_args()
    device = torch.device("cuda:0")
    accs = []
    for k in range(args.seeds):
        seed = args.seed0 + k
        t0 = time.time()
        if args.model == "lds":
            res = run_lds(args.dataset, seed, device, pretrain=not args.no_pretrain, tau=args.tau, fused=args.fused)
            res["path"] = "fused engine" if args.fused else "drop-in autograd"
        else:
            res = run_gcn(args.dataset, seed, device)
        res.update(seed=seed, seconds=time.time() - t0, dataset=args.dataset, model=args.model)
        accs.append(100.0 * res["acc.test.final"])
        print(json.dumps(res), flush=True)
    pub = PUBLISHED.get((args.model, args.dataset))
    print(json.dumps({"summary": f"{args.model} {args.dataset}", "runs": len(accs), "test_acc_mean": float(np.mean(accs)),
                      "test_acc_std": float(np.std(accs)), "published": pub,
                      "config": f"LDS (τ={args.tau}, patience 20, S_eval 16, θ lr 0.1 decay 0.99, "
                                f"{'no pretrain' if args.no_pretrain else 'pretrain'}, "
                                f"{'fused engine' if args.fused else 'drop-in autograd'})"
                      if args.model == "lds" else "GCN (Adam 0.01, wd 5e-4, 200 epochs, patience 10)"}), flush=True)


if __name__ == "__main__":
    main()
