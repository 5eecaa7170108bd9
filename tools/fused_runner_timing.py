"""FusedBilevelRunner.train wall time at Cora shape (synthetic, kNN θ₀),
per-step HIP graphs on vs off, fixed epoch budget (patience large so both
runs take the same steps).  Prints one JSON line."""
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


def run(step_graphs, inner_max, outer_max):
    args = argparse.Namespace(dataset="cora", seed=1, samples=1, graph_model="lds", tau=5, path="engine")
    data, runner, _ = bench.build(args, 0, torch.device("cuda:0"))
    fr = FusedBilevelRunner(runner.inner_trainer, runner.outer_trainer, runner.data, n_samples_empirical_mean=16,
                            step_graphs=step_graphs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fr.train(patience=1000, hyper_gradient_interval=5, inner_loop_max_epochs=inner_max,
             outer_loop_max_epochs=outer_max)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return dt, fr.inner_steps, fr.evaluate()


def main():
    inner_max, outer_max = 100, 3
    out = {"workload": f"cora-shaped FusedBilevelRunner.train, tau=5, inner max {inner_max}, outer max {outer_max}"}
    for sg in (False, True):
        dt, steps, ev = run(sg, inner_max, outer_max)
        out["step_graphs" if sg else "eager"] = {"seconds": dt, "inner_steps": steps,
                                                 "ms_per_inner_step": 1000.0 * dt / steps,
                                                 "val_loss_final": ev["loss.val.final"]}
    out["speedup"] = out["eager"]["seconds"] / out["step_graphs"]["seconds"]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
