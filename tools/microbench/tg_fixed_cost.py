"""Where the Cora θ-grad's fixed cost goes (form 10, lds_theta_grad_direct,
mode 2, no dθ store as in the bench): µs per launch as a dependent chain of
20 copies in one HIP graph, with and without the next window's six-graph
draw, at k = 264 (17 chunks) and k = 16 (one chunk).  Run once per library
(LDSGNN_LIB): the product, and timing-only builds of thetagrad.hip with
tools/microbench/tg_fixed_cost.patch applied (`git apply`, against the
thetagrad.hip of commit 2bccbf0) and
-DLDS_TG_EXPT=1 (no θ preload), 2 (no k-loop), 3 (no θ store), 5 (θ loaded
after the k-loop), 6 (no in-loop ring refill), 7 (no MFMAs), 8 (refill kept,
no load wait) — their results are wrong by construction; with
LDS_TG_EXPT=0 the patch is the product with the refill pieces threaded
through the second half's MFMAs (bit-identical, measured and not kept).
Results: profiles/r06_theta_fixed_cost.jsonl, DESIGN.md §4i (round 6).
Usage (GPU box): LDSGNN_LIB=... python tools/microbench/tg_fixed_cost.py LABEL"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lds-gnn_amd")]
import torch  # noqa: E402

import ldsgnn  # noqa: E402,F401
from ldsgnn import _native as nat  # noqa: E402
from ldsgnn.rng import TAG_GRAPH, tag_for  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from tg_draw_ab import chain_us  # noqa: E402


def run(label, n, k, graphs):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(n + k)
    u = torch.randn((n, k), generator=g, device=dev) * 0.01
    v = torch.randn((n, k), generator=g, device=dev) * 0.01
    r = torch.randn(n, generator=g, device=dev) * 0.01
    theta = torch.rand(n * (n + 1) // 2, generator=g, device=dev)
    scal = torch.zeros(64, dtype=torch.uint8, device=dev)
    scal[16:24].view(torch.float64).fill_(1e-9)
    words = nat.lib.lds_bitmask_words(n)
    wsi = nat.lib.lds_sample_ws_ints(n)
    base = torch.zeros(4, dtype=torch.int32, device=dev)
    bits = torch.zeros((max(graphs, 1), n, words), dtype=torch.int64, device=dev)
    deg = torch.zeros((max(graphs, 1), wsi), dtype=torch.int32, device=dev)
    ne = nat.lib.lds_planes_t128_elems(n, k)
    up = torch.empty(ne, dtype=torch.int16, device=dev)
    vp = torch.empty(ne, dtype=torch.int16, device=dev)
    st = nat.stream_of(dev)
    nat.call("lds_split_planes_t128", nat.ptr(u), n, k, k, nat.ptr(up), st)
    nat.call("lds_split_planes_t128", nat.ptr(v), n, k, k, nat.ptr(vp), st)

    def direct():
        nat.call("lds_theta_grad_direct", nat.ptr(up), nat.ptr(vp), k, nat.ptr(r), 1, n, 1, nat.ptr(theta), n,
                 None, 2, nat.ptr(scal), 1.0, 99, tag_for(TAG_GRAPH, 0), nat.ptr(base), 0, graphs, nat.ptr(bits),
                 words, nat.ptr(deg), nat.stream_of(dev))
        if graphs:
            deg.zero_()

    zt = chain_us(lambda: deg.zero_(), dev) if graphs else 0.0
    t = min(chain_us(direct, dev) for _ in range(3)) - zt
    print(json.dumps({"lib": label, "n": n, "k": k, "graphs": graphs, "chain_us": round(t, 2)}), flush=True)


def main():
    label = sys.argv[1] if len(sys.argv) > 1 else "product"
    for k in (264, 16):
        for graphs in (0, 6):
            run(label, 2708, k, graphs)


if __name__ == "__main__":
    main()
