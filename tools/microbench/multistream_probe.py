"""Probe: do S independent engine windows (one HIP graph each) replayed on S
streams overlap on MI355X?  Prints inner steps/s per sample count for
(a) one stream, graphs back to back, (b) one stream per engine."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (ROOT, os.path.join(ROOT, "lds-gnn_amd")):
    sys.path.insert(0, p)
import numpy as np
import torch

import ldsgnn
from ldsgnn.data.synthetic import knn_init, make_dataset
from ldsgnn.engine import LdsEngine
from ldsgnn.rng import Generator
from ldsgnn.utils.graph import split_mask

dev = torch.device("cuda:0")
data = knn_init(make_dataset("cora", seed=1), k=10)
np.random.seed(1)
data.val_mask, opt_mask = split_mask(data.val_mask, 0.5, shuffle=True)
data = data.to(dev)
from oracle import lds_oracle as O  # noqa: E402  (only for get_triu_values)
theta0 = O.get_triu_values(data.dense_adj.cpu()).to(dev)
tau = 5
W = 40
for S in (1, 2, 4, 8, 16):
    engs, streams = [], []
    for s in range(S):
        torch.manual_seed(s)
        e = LdsEngine(data.x, data.y, data.train_mask, opt_mask.to(dev), theta0.clone(), data.num_classes,
                      outer_lr=0.1, lr_decay=0.99, tau=tau, generator=Generator(7, s))
        e.inner_step(); e.hyper_step()
        e.capture_window(tau)
        engs.append(e)
        streams.append(torch.cuda.Stream(dev))
    torch.cuda.synchronize()
    for mode in ("serial", "streams"):
        def run(windows):
            main = torch.cuda.current_stream(dev)
            for _ in range(windows):
                if mode == "serial":
                    for e in engs:
                        e.replay(1)
                else:
                    ev = torch.cuda.Event()
                    ev.record(main)
                    for e, st in zip(engs, streams):
                        st.wait_event(ev)
                        with torch.cuda.stream(st):
                            e.replay(1)
                    for st in streams:
                        main.wait_stream(st)
        run(4)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(W)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"S={S:2d} {mode:8s} sample-steps/s {S * W * tau / dt:10.0f}  window {1e6 * dt / W:8.1f} us", flush=True)
