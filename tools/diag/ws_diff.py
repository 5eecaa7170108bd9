"""Where the persistent θ-grad form's draw differs from form 10's (debug aid):
graphs, rows and 64-column words whose bits differ, per tile position."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lds-gnn_amd")]
import torch  # noqa: E402

import ldsgnn  # noqa: E402,F401
from ldsgnn import _native as nat  # noqa: E402
from ldsgnn.rng import TAG_GRAPH, tag_for  # noqa: E402


def main(n=4100, k=264, graphs=6):
    device = "cuda"
    g = torch.Generator().manual_seed(n + k + graphs)
    u = torch.randn(n, k, generator=g).to(device)
    v = (torch.randn(n, k, generator=g) * 0.3).to(device)
    r = torch.randn(n, generator=g).to(device)
    theta = (torch.rand(n * (n + 1) // 2, generator=g) * 1.2 - 0.1).to(device)
    scal = torch.zeros(64, dtype=torch.uint8, device=device)
    scal[16:24].view(torch.float64).fill_(0.05)
    st = nat.stream_of(torch.device(device))
    words = nat.lib.lds_bitmask_words(n)
    wsi = nat.lib.lds_sample_ws_ints(n)
    base = torch.tensor([5, 0, 0, 0], dtype=torch.int32, device=device)
    seed, tag, off = 777, tag_for(TAG_GRAPH, 1), 3
    ne = nat.lib.lds_planes_t128_elems(n, k)
    up = torch.empty(ne, dtype=torch.int16, device=device)
    vp = torch.empty(ne, dtype=torch.int16, device=device)
    nat.call("lds_split_planes_t128", nat.ptr(u), n, k, k, nat.ptr(up), st)
    nat.call("lds_split_planes_t128", nat.ptr(v), n, k, k, nat.ptr(vp), st)
    hf = int(nat.lib.lds_theta_grad_ws_floats())
    handoff = torch.full((hf,), float("nan"), device=device)
    res = []
    for ws in (False, True):
        th = theta.clone()
        bits = torch.zeros((graphs, n, words), dtype=torch.int64, device=device)
        deg = torch.zeros((graphs, wsi), dtype=torch.int32, device=device)
        if ws:
            nat.call("lds_theta_grad_direct_ws", nat.ptr(up), nat.ptr(vp), k, nat.ptr(r), 1, 1, 1, nat.ptr(th), n, 0,
                     nat.ptr(scal), 0.5, seed, tag, nat.ptr(base), off, graphs, nat.ptr(bits), words, nat.ptr(deg),
                     nat.ptr(handoff), hf, st)
        else:
            nat.call("lds_theta_grad_direct", nat.ptr(up), nat.ptr(vp), k, nat.ptr(r), 1, 1, 1, nat.ptr(th), n, 0,
                     2, nat.ptr(scal), 0.5, seed, tag, nat.ptr(base), off, graphs, nat.ptr(bits), words,
                     nat.ptr(deg), st)
        torch.cuda.synchronize()
        res.append((th, bits, deg))
    (ta, ba, da), (tb, bb, db) = res
    out = {"theta_equal": bool(torch.equal(ta, tb))}
    d = (ba != bb)
    out["words_differ"] = int(d.sum())
    out["graphs_differ"] = [int(x) for x in d.flatten(1).any(1).nonzero().flatten()]
    idx = d.nonzero()
    if idx.numel():
        rows = idx[:, 1]
        wds = idx[:, 2]
        out["rows_first"] = [int(x) for x in rows[:20]]
        out["words_first"] = [int(x) for x in wds[:20]]
        out["row_tiles"] = sorted({int(x) // 128 for x in rows})[:40]
        out["col_tiles"] = sorted({int(x) // 2 for x in wds})[:40]
        # xor popcount of differing words
        x = (ba ^ bb)[d]
        out["bits_differ"] = int(sum(bin(int(w) & (2**64 - 1)).count("1") for w in x[:2000]))
        out["sample"] = [[int(a) & (2**64 - 1), int(b) & (2**64 - 1)] for a, b in zip(ba[d][:5], bb[d][:5])]
    out["deg_equal"] = bool(torch.equal(da, db))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
