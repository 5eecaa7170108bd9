"""How much of θ sits exactly on the clamp bounds {0, 1} during the bench
workload (Cora, sklearn kNN θ₀, τ = 5, S = 1), by window: the fraction of
entries, of 4-row quads (one Philox call's outputs) and of 16 × 64 blocks
(one wave's draw work) whose draws are decided without a uniform.
Usage (GPU box): python tools/diag/theta_stats.py [windows...]"""
import json
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lds-gnn_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


def stats(theta, n):
    iu = torch.triu_indices(n, n, device=theta.device)
    full = torch.full((n, n), 0.5, device=theta.device)
    full[iu[0], iu[1]] = theta
    full.diagonal().fill_(0.0)  # the diagonal is never drawn
    decided = (full == 0) | (full == 1)
    upper = torch.triu(torch.ones(n, n, dtype=torch.bool, device=theta.device), 1)
    out = {"frac_zero": float(((full == 0) & upper).sum() / upper.sum()),
           "frac_one": float(((full == 1) & upper).sum() / upper.sum())}
    nq = n // 64 * 64
    d = decided[:nq, :nq] | ~upper[:nq, :nq]
    quads = d.view(nq // 4, 4, nq).all(1)
    out["frac_quads_decided"] = float(quads.float().mean())
    blocks = d.view(nq // 16, 16, nq // 64, 64).all(3).all(1)
    out["frac_16x64_blocks_decided"] = float(blocks.float().mean())
    return out


def main():
    checkpoints = [int(a) for a in sys.argv[1:]] or [0, 4, 20, 100, 400]
    args = types.SimpleNamespace(samples=1, dataset="cora", seed=597905255 % (2 ** 31), graph_model="lds")
    dev = torch.device("cuda:0")
    data, runner, _ = bench.build(args, 0, dev)
    eng, _ = bench.make_engine(runner, 5, 1)
    eng.inner_step()
    eng.hyper_step()
    eng.capture_window(5, windows=1, prefetch=True)
    done = 0
    for c in sorted(checkpoints):
        eng.replay(c - done)
        done = c
        torch.cuda.synchronize()
        print(json.dumps({"window": c, **stats(eng.theta, data.num_nodes)}), flush=True)


if __name__ == "__main__":
    main()
