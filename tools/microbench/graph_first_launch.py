"""First replay of a captured window group against later ones (the bench's
timed region replays the 4-window graph for the first time when warmup is a
single window): wall time of replay(4) right after capture, then again,
without and with lds_graph_upload (hipGraphUpload) of the sealed graphs.
Usage (GPU box): python tools/microbench/graph_first_launch.py"""
import json
import os
import sys
import time
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lds-gnn_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from ldsgnn import _native as nat  # noqa: E402


def timed(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return 1e6 * (time.perf_counter() - t0)


def main():
    dev = torch.device("cuda:0")
    args = SimpleNamespace(samples=1, dataset="cora", seed=0, graph_model="lds", gae_dropout=0.0)
    _, runner, _ = bench.build(args, 0, dev)
    eng, _ = bench.make_engine(runner, 5, 1)
    eng.inner_step()
    eng.hyper_step()
    for upload in (False, True, False, True):
        nat.UPLOAD_GRAPHS = upload
        eng.capture_window(5, windows=4, prefetch=True)
        eng.replay(1)  # the bench's warmup: one window on the 1-window graph
        us = [timed(lambda: eng.replay(4)) for _ in range(4)]
        print(json.dumps({"upload": upload, "replay4_us": [round(u, 1) for u in us]}), flush=True)


if __name__ == "__main__":
    main()
