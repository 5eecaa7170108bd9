"""How much of θ is exactly zero while the bench workload trains (Cora, kNN
θ₀, τ = 5, one sample): entries whose draw threshold ceil(θ·2^24) is 0 need
no random word (the edge is never drawn).  Reports, after 0 .. 2000 replayed
windows, the fraction of zero entries of the strict upper triangle and the
fraction of aligned blocks that are zero throughout, for the two Philox
footprints of a wave in the draw epilogues (4 rows × 64 columns: the 64-tile
sampler; 8 rows × 32 columns: the eight-wave 128-tile θ-grad epilogue).
Usage (GPU box): python tools/microbench/theta_zero_census.py [dataset]"""
import json
import os
import sys
from types import SimpleNamespace

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lds-gnn_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


def census(theta, n):
    """Zero fractions of the packed upper triangle θ (diagonal included)."""
    iu = torch.triu_indices(n, n, device=theta.device)
    dense = torch.zeros((n, n), dtype=torch.bool, device=theta.device)
    dense[iu[0], iu[1]] = theta > 0  # nonzero threshold
    dense &= torch.ones((n, n), dtype=torch.bool, device=theta.device).triu(1)
    upper = n * (n - 1) // 2
    out = {"nonzero_frac": float(dense.sum()) / upper}
    for rows, cols in ((4, 64), (8, 32)):
        nr, nc = (n + rows - 1) // rows, (n + cols - 1) // cols
        pad = torch.zeros((nr * rows, nc * cols), dtype=torch.bool, device=theta.device)
        pad[:n, :n] = dense
        blk = pad.view(nr, rows, nc, cols).any(3).any(1)  # block holds a nonzero threshold
        # blocks that touch the strict upper triangle
        bi = torch.arange(nr, device=theta.device)[:, None] * rows
        bj = torch.arange(nc, device=theta.device)[None, :] * cols + cols - 1
        live = bj > bi
        out[f"blocks_{rows}x{cols}_nonzero_frac"] = float((blk & live).sum()) / float(live.sum())
    return out


def main():
    dataset = sys.argv[1] if len(sys.argv) > 1 else "cora"
    dev = torch.device("cuda:0")
    args = SimpleNamespace(samples=1, dataset=dataset, seed=0, graph_model="lds", gae_dropout=0.0)
    data, runner, opt_mask = bench.build(args, 0, dev)
    eng, _ = bench.make_engine(runner, 5, 1)
    eng.capture_window(5, windows=4, prefetch=True)
    done = 0
    for target in (0, 10, 100, 500, 2000):
        eng.replay(target - done)
        done = target
        torch.cuda.synchronize()
        rec = {"dataset": dataset, "windows": done, **census(eng.theta, eng.n)}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
