"""Debug: batched-engine mean hypergradient vs oracle replicas, per hyper step."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "lds-gnn_amd")):
    sys.path.insert(0, p)
import torch
from oracle import lds_oracle as O
import tests.parity_harness as H

orig = O.replica_hyper_step
store = {}
def spy(problems):
    res = [p.hyper_grad() for p in problems]
    g = res[0][2].clone()
    for r in res[1:]:
        g += r[2]
    g /= len(problems)
    for p in problems:
        p.apply_hyper_update(g)
    store.setdefault("ind", []).append([float(r[2].abs().max()) for r in res])
    store.setdefault("g", []).append(g)
    return [(r[0], r[1]) for r in res], g
O.replica_hyper_step = spy
for (S, tau, dp) in [(3, 5, 0.5), (4, 1, 0.0), (2, 5, 0.0), (1, 5, 0.5)]:
    store.clear()
    res = H.run_engine_samples_and_oracle(samples=S, n=110, f_in=26, classes=5, steps=11, tau=tau, dropout=dp,
                                          seed=7, replica0=2)
    print(S, tau, dp, {k: v for k, v in res.items() if k.startswith("max")}, "ind max", store["ind"][:3],
          "mean max", [float(g.abs().max()) for g in store["g"][:3]], flush=True)
