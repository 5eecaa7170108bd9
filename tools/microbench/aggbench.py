"""Time aggregation-kernel variants (tools/microbench/aggbench.hip) in a
replayed chain of K dependent launches (ping-pong Z -> Y -> Z) on the bench
graphs: the real Cora kNN θ₀ graph (config 2), the given Cora graph (config 1)
and the synthetic Cora-shaped kNN graph.  Prints one JSON line per
(graph, variant) with µs per launch and the max deviation from variant 0."""
import ctypes
import json
import os
import subprocess
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "lds-gnn_amd")]
import torch  # noqa: E402

from ldsgnn import ops  # noqa: E402
from ldsgnn.data.workloads import load_workload  # noqa: E402
from ldsgnn.rng import Generator  # noqa: E402
from ldsgnn.utils.graph import get_triu_values  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libaggbench.so")


def load():
    lib = ctypes.CDLL(LIB)
    lib.aggbench_launch.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_int] + [ctypes.c_void_p] * 3
    lib.aggbench_launch_plan.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 3
    return lib


def ell_of(g):
    n = g.n
    rp = g.row_ptr.long()
    deg = rp[1:] - rp[:-1]
    k = torch.arange(16, device=rp.device)
    pos = rp[:-1, None] + k[None, :]
    valid = k[None, :] < deg[:, None]
    j = torch.where(valid, g.col.long()[pos.clamp(max=g.col.numel() - 1)], torch.arange(n, device=rp.device)[:, None])
    sv = torch.where(valid, g.s[j], torch.zeros_like(g.s[j]))
    return torch.stack([j.int(), sv.view(torch.int32)], -1).contiguous()


def main(K=200):
    lib = load()
    dev = torch.device("cuda:0")
    out = []
    for wl in ("cora", "cora-given", "cora-synthetic"):
        data = load_workload(wl, device=dev)
        n = data.num_nodes
        g = ops.sample_graph_from_triu(get_triu_values(data.dense_adj).contiguous(), n, generator=Generator(1),
                                       track_grad=False)
        ell = ell_of(g)
        deg = (g.row_ptr[1:] - g.row_ptr[:-1])
        z0 = torch.randn(n, 16, device=dev)
        ref = None
        heavy = deg > 64
        idx = torch.arange(n, device=dev)
        plan = torch.cat([idx[heavy], idx[~heavy]]).int().contiguous()
        nh = int(heavy.sum())

        def launch(v, src, dst, st):
            if v == 4:
                return lib.aggbench_launch_plan(g.row_ptr.data_ptr(), g.col.data_ptr(), g.s.data_ptr(),
                                                plan.data_ptr(), nh, n, src.data_ptr(), dst.data_ptr(), st)
            return lib.aggbench_launch(v, g.row_ptr.data_ptr(), g.col.data_ptr(), g.s.data_ptr(), ell.data_ptr(), n,
                                       src.data_ptr(), dst.data_ptr(), st)

        for v in (8, 9, 0, 1, 2, 3, 4):
            y = torch.empty_like(z0)
            st = torch.cuda.current_stream().cuda_stream
            assert launch(v, z0, y, st) == 0
            torch.cuda.synchronize()
            if v == 0:
                ref = y.clone()
            err = float((y - ref).abs().max() / ref.abs().max()) if v in (0, 1, 2, 3, 4) else None
            a, b = z0.clone(), torch.empty_like(z0)
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.stream(s):
                with torch.cuda.graph(gr, stream=s):
                    for i in range(K):
                        src, dst = (a, b) if i % 2 == 0 else (b, a)
                        launch(v, src, dst, s.cuda_stream)
            torch.cuda.current_stream().wait_stream(s)
            gr.replay()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                gr.replay()
            torch.cuda.synchronize()
            us = (time.perf_counter() - t0) / (5 * K) * 1e6
            row = {"graph": wl, "variant": v, "us_per_launch": us, "rel_err_vs_v0": err,
                   "max_deg": int(deg.max()), "mean_deg": float(deg.float().mean())}
            print(json.dumps(row), flush=True)
            out.append(row)


if __name__ == "__main__":
    main()
