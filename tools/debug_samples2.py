"""Debug: single-chain engine vs oracle for replicas 2..4 (conditioning check)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "lds-gnn_amd")):
    sys.path.insert(0, p)
import tests.parity_harness as H
for r0 in (2, 3, 4):
    res = H.run_engine_samples_and_oracle(samples=1, n=110, f_in=26, classes=5, steps=11, tau=5, dropout=0.5,
                                          seed=7, replica0=r0)
    print("replica", r0, {k: v for k, v in res.items() if k.startswith("max")}, flush=True)
for S, r0 in ((2, 2), (2, 3), (3, 2)):
    res = H.run_engine_samples_and_oracle(samples=S, n=110, f_in=26, classes=5, steps=1, tau=5, dropout=0.5,
                                          seed=7, replica0=r0)
    print("S", S, "r0", r0, "1 step", {k: v for k, v in res.items() if k.startswith("max")}, flush=True)
