"""How often the sampler's Philox draw decides nothing: the fraction of
(column, row-quad) cells whose four θ entries are all <= 0 or >= 1 (the
Bernoulli outcome is fixed whatever u is), per cell and per wave (64 columns ×
one quad), over the bench's real-Cora training trajectory.
Usage (GPU box): python tools/diag/theta_quads.py > gpurun_out/theta_quads.jsonl"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "lds-gnn_amd"))
import bench  # noqa: E402


def quad_stats(theta, n):
    iu = torch.triu_indices(n, n, device=theta.device)
    dense = torch.full((n, n), -1.0, device=theta.device)
    dense[iu[0], iu[1]] = theta
    dense.fill_diagonal_(-1.0)  # the strict upper triangle only (the tile kernel's -1 marks)
    dense = torch.where(torch.arange(n, device=theta.device)[:, None] < torch.arange(n, device=theta.device)[None, :],
                        dense, torch.full_like(dense, -1.0))
    npad = (n + 63) // 64 * 64
    d = torch.full((npad, npad), -1.0, device=theta.device)
    d[:n, :n] = dense
    det = (d <= 0) | (d >= 1)
    quad = det.view(npad // 4, 4, npad).all(1)                   # [row quad, column]
    # only cells of the upper-triangle tiles (bi <= bj) are drawn
    rb = torch.arange(npad // 4, device=theta.device)[:, None] * 4 // 64
    cb = torch.arange(npad, device=theta.device)[None, :] // 64
    drawn = rb <= cb
    wave = quad.view(npad // 4, npad // 64, 64).all(2)           # 64 columns of one quad
    wdrawn = drawn.view(npad // 4, npad // 64, 64)[:, :, 0]
    zero = ((d > 0) & (d < 1)).float().sum() / (n * (n - 1) / 2)
    return {"cells_fixed": float(quad[drawn].float().mean()), "waves_fixed": float(wave[wdrawn].float().mean()),
            "frac_open_entries": float(zero)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--windows", type=int, default=400)
    a = ap.parse_args()
    args = argparse.Namespace(dataset="cora", seed=597905255 % (2 ** 31), samples=1, graph_model="lds", tau=5)
    dev = torch.device("cuda", 0)
    data, runner, opt_mask = bench.build(args, 0, dev)
    eng, _ = bench.make_engine(runner, 5, 1)
    eng.inner_step()
    eng.hyper_step()
    eng.capture_window(5)
    done = 0
    for target in (0, 10, 50, 100, 200, a.windows):
        if target > done:
            eng.replay(target - done)
            done = target
        torch.cuda.synchronize()
        print(json.dumps({"window": done, **quad_stats(eng.theta, eng.n)}), flush=True)


if __name__ == "__main__":
    main()
