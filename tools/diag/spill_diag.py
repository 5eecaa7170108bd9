"""Spill-pass CSR-SpMM (dbg 23) against the row-block kernel (dbg 22) on
small random CSR: which rows differ and by how many neighbours per column
residue (z[j, f] = [j % 16 == f], s = 1: y counts a row's neighbours per
residue).  Usage (GPU box): python tools/diag/spill_diag.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lds-gnn_amd")]
import torch  # noqa: E402

import ldsgnn  # noqa: E402,F401
from ldsgnn import _native as nat  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "tools", "variants"))
import variants  # noqa: E402  (the tools-only variants library)


def run(n, dens, grid, seed):
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(seed)
    a = torch.rand(n, n, generator=g) < dens
    rows, cols = a.nonzero(as_tuple=True)
    rp = torch.zeros(n + 1, dtype=torch.int64)
    rp[1:] = torch.cumsum(a.sum(1), 0)
    rpd, cold = rp.int().to(dev), cols.int().to(dev)
    s = torch.ones(n, device=dev)
    z = torch.zeros(n, 16)
    z[torch.arange(n), torch.arange(n) % 16] = 1.0
    z = z.to(dev)
    ws = torch.empty(variants.ws_bytes(n), dtype=torch.uint8, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    y = {}
    for name, dbg in (("rowblock", 22), ("spill", 23), ("spill_d6", 33), ("spill_d12", 34), ("spill_vm0", 35), ("rowblock_hybrid", 6), ("spill_quad", 36), ("spill_win", 37), ("spill_win_d6", 38), ("spill_ahead", 39), ("spill_rolled", 41), ("spill_rolled_d12", 42), ("spill_ns12_d5", 43), ("spill_ns12_d6", 44), ("ns12_d4", 45), ("ns12_d5_win", 46), ("ns12_d3", 47), ("ns14_d4", 48), ("ns14_d3", 49), ("ns12_d4_fq", 50), ("ns14_d4_fq", 51), ("ns12_d4_fs", 52), ("ns12_d3_fs", 53), ("e8_d3", 54), ("e8_d2", 55), ("e8_d2_ns8", 56), ("e8_d2_ns14", 57), ("reg3", 60), ("reg4", 61), ("reg6", 62), ("reg4_dyn", 63), ("reg4_cache", 64), ("reg4_lean", 65), ("reg4_ballot", 66), ("reg4_ns14", 67), ("e12_d3", 68), ("e12_d4", 69)):
        out = torch.empty(n, 16, device=dev)
        if dbg == 22:
            nat.call("lds_spmm_norm_dense", nat.ptr(rpd), nat.ptr(cold), nat.ptr(s), n, nat.ptr(z), 16, nat.ptr(out),
                     16, 0, nat.ptr(ws), -256, 1, nat.ptr(err), nat.stream_of(dev))
        variants.spmm_dense(nat.ptr(rpd), nat.ptr(cold), nat.ptr(s), n, nat.ptr(z), 16, nat.ptr(out),
                            16, nat.ptr(ws), dbg, nat.stream_of(dev))
        torch.cuda.synchronize()
        y[name] = out.cpu().round().long()
    ref = torch.zeros(n, 16, dtype=torch.long)
    ref.index_add_(0, rows, torch.nn.functional.one_hot(cols % 16, 16))
    bad = {k: (v != ref).any(1).nonzero().flatten().tolist() for k, v in y.items()}
    out = {"n": n, "dens": dens, "grid": grid, "seed": seed, "nnz": int(rp[-1]),
           "bad_rows": {k: v[:20] for k, v in bad.items()}, "bad_count": {k: len(v) for k, v in bad.items()}}
    for r in bad["spill"][:5]:
        out[f"row{r}"] = {"deg": int(rp[r + 1] - rp[r]), "start": int(rp[r]),
                          "diff": (y["spill"][r] - ref[r]).tolist()}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    for n, dens, seed in ((1500, 0.5, 1), (700, 0.9, 3), (6000, 0.3, 5), (12000, 0.2, 7)):
        run(n, dens, 0, seed)
