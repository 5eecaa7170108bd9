"""The embedding graph model (P = σ(E·Eᵀ), 16-dim E, init ±0.001: P ≈ 0.5,
dense sampled graphs) and the GAE model (factory defaults) at Cora shape: inner steps/s of the drop-in trainers
against FusedBilevelRunner (inner loop + dθ on the engine, long-row bitmask
aggregation; outer SGD on E by autograd through P).  Fixed epoch budget;
one JSON line."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "lds-gnn_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402

import bench  # noqa: E402
from ldsgnn.fused import FusedBilevelRunner  # noqa: E402


def run(fused, inner_max, outer_max, model="embedding"):
    args = argparse.Namespace(dataset="cora", seed=1, samples=1, graph_model=model, tau=5, path="autograd")
    data, runner, _ = bench.build(args, 0, torch.device("cuda:0"))
    if fused:
        runner = FusedBilevelRunner(runner.inner_trainer, runner.outer_trainer, runner.data,
                                    n_samples_empirical_mean=16)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    runner.train(patience=1000, hyper_gradient_interval=5, inner_loop_max_epochs=inner_max,
                 outer_loop_max_epochs=outer_max)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    steps = runner.inner_steps if fused else None
    return dt, steps


def main():
    inner_max, outer_max = 60, 2
    for model in ("embedding", "gae"):
        out = {"workload": f"cora-shaped {model} model, tau=5, inner max {inner_max}, outer max {outer_max} "
                           "(second of two runs each: one-time setup excluded)"}
        for fused in (True, False):
            run(fused, 5, 0, model)
            dt, steps = run(fused, inner_max, outer_max, model)
            out["fused" if fused else "dropin"] = {"seconds": dt}
            if steps:
                out["inner_steps"] = steps
        out["speedup"] = out["dropin"]["seconds"] / out["fused"]["seconds"]
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
