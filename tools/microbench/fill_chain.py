"""The window fill (lds_sample_fill_csr: CSR, s and the ELL head from drawn
bits and degree counts) for 1 and for 6 Cora-sized graphs, each as a
dependent chain of 20 copies in one HIP graph: is the fill's time per launch
its workgroups' latency (1 graph costs about what 6 do) or its work (1 graph
about a sixth)?  θ ~ U(0, 0.0125) gives ≈17 entries per row, as the sampled
Cora graphs.  One JSON line.
Usage (GPU box): python tools/microbench/fill_chain.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lds-gnn_amd")]
import torch  # noqa: E402

import ldsgnn  # noqa: E402,F401
from ldsgnn import _native as nat  # noqa: E402
from ldsgnn.rng import TAG_GRAPH, tag_for  # noqa: E402
from tg_draw_ab import chain_us  # noqa: E402


def main():
    n, count = 2708, 6
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(5)
    theta = torch.rand(n * (n + 1) // 2, generator=g, device=dev) * 0.0125
    words = nat.lib.lds_bitmask_words(n)
    wsi = nat.lib.lds_sample_ws_ints(n)
    cap = 4 * 64 * n
    base = torch.zeros(4, dtype=torch.int32, device=dev)
    bits = torch.zeros((count, n, words), dtype=torch.int64, device=dev)
    deg = torch.zeros((count, wsi), dtype=torch.int32, device=dev)
    rp = torch.zeros((count, n + 1), dtype=torch.int32, device=dev)
    col = torch.zeros((count, cap), dtype=torch.int32, device=dev)
    s = torch.zeros((count, n), dtype=torch.float32, device=dev)
    ell = torch.zeros((count, n * 128), dtype=torch.int32, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    st = nat.stream_of(dev)
    nat.call("lds_sample_graphs_multi", nat.ptr(theta), n, 11, tag_for(TAG_GRAPH, 0), 1, nat.ptr(base), 0, count, 1,
             nat.ptr(bits), words, nat.ptr(deg), nat.ptr(rp), nat.ptr(col), cap, nat.ptr(s), nat.ptr(ell), 0, 1,
             nat.ptr(err), st)
    torch.cuda.synchronize()
    out = {"n": n, "entries_per_graph": int(rp[0, n].item()), "err": int(err.item())}
    for k in (1, 2, 6):
        def fill(k=k):
            nat.call("lds_sample_fill_csr", nat.ptr(bits), n, words, nat.ptr(deg), k, nat.ptr(rp), nat.ptr(col), cap,
                     nat.ptr(s), nat.ptr(ell), 0, nat.ptr(err), nat.stream_of(dev))  # (the capture stream)
        out[f"fill_{k}_graphs_us"] = chain_us(fill, dev)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
