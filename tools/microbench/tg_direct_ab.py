"""θ-grad form 10 (direct-staged eight-wave 128-tile on pre-split planes,
lds_theta_grad_direct) against form 9 (the eight-wave 128-tile that splits
while staging) and the by-shape default, at the engine's shapes: identical θ /
dθ / bits / degrees, then µs per launch as a dependent chain of 20 copies in
one HIP graph (HIP events on the launch stream), with and without the next
window's draw; the plane split (lds_split_planes_t128, U and V) timed alone.
Usage (GPU box): python tools/microbench/tg_direct_ab.py [cora|s16|c5|graphs|all]"""
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
from tg_draw_ab import BF16_PEAK_TF, chain_us  # noqa: E402

FORM9, FORM_BY_SHAPE = 9, 1


def run(name, n, k, graphs):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(n + k)
    u = torch.randn((n, k), generator=g, device=dev) * 0.01
    v = torch.randn((n, k), generator=g, device=dev) * 0.01
    r = torch.randn(n, generator=g, device=dev) * 0.01
    theta0 = torch.rand(n * (n + 1) // 2, generator=g, device=dev) * 0.02
    theta = theta0.clone()
    grad = torch.empty_like(theta)
    scal = torch.zeros(64, dtype=torch.uint8, device=dev)
    scal[16:24].view(torch.float64).fill_(1e-6)
    words = nat.lib.lds_bitmask_words(n)
    wsi = nat.lib.lds_sample_ws_ints(n)
    base = torch.zeros(4, dtype=torch.int32, device=dev)
    bits = torch.zeros((graphs, n, words), dtype=torch.int64, device=dev)
    deg = torch.zeros((graphs, wsi), dtype=torch.int32, device=dev)
    ne = nat.lib.lds_planes_t128_elems(n, k)
    up = torch.empty(ne, dtype=torch.int16, device=dev)
    vp = torch.empty(ne, dtype=torch.int16, device=dev)
    seed, tag = 99, tag_for(TAG_GRAPH, 0)
    flop = 24.0 * k * n * (n + 1) / 2
    out = {"workload": name, "n": n, "k": k, "graphs": graphs}

    def split():
        nat.call("lds_split_planes_t128", nat.ptr(u), n, k, k, nat.ptr(up), nat.stream_of(dev))
        nat.call("lds_split_planes_t128", nat.ptr(v), n, k, k, nat.ptr(vp), nat.stream_of(dev))

    split()

    def plain(form):
        nat.call("lds_theta_grad_ex", nat.ptr(u), nat.ptr(v), k, k, nat.ptr(r), 1, n, 1, nat.ptr(theta), n,
                 nat.ptr(grad), 2, nat.ptr(scal), 1.0, form, nat.stream_of(dev))

    def direct(gr):
        nat.call("lds_theta_grad_direct", nat.ptr(up), nat.ptr(vp), k, nat.ptr(r), 1, n, 1, nat.ptr(theta), n,
                 nat.ptr(grad), 2, nat.ptr(scal), 1.0, seed, tag, nat.ptr(base), 0, gr, nat.ptr(bits), words,
                 nat.ptr(deg), nat.stream_of(dev))

    def drawcall(form):
        nat.call("lds_theta_grad_sgd_draw", nat.ptr(u), nat.ptr(v), k, k, nat.ptr(r), 1, 1, nat.ptr(theta), n,
                 nat.ptr(grad), nat.ptr(scal), seed, tag, nat.ptr(base), 0, graphs, nat.ptr(bits), words,
                 nat.ptr(deg), form, nat.stream_of(dev))

    def state(fn):
        theta.copy_(theta0)
        bits.zero_()
        deg.zero_()
        fn()
        torch.cuda.synchronize()
        return theta.clone(), grad.clone(), bits.clone(), deg.clone()

    ref_plain = state(lambda: plain(FORM9))
    out["plain_identical"] = all(bool(torch.equal(a, b)) for a, b in zip(ref_plain[:2], state(lambda: direct(0))[:2]))
    for label, fn in (("plain_form9", lambda: plain(FORM9)), ("plain_by_shape", lambda: plain(FORM_BY_SHAPE)),
                      ("plain_form10", lambda: direct(0))):
        t = chain_us(fn, dev)
        out[label] = {"chain_us": t, "bf16_frac": flop / t / 1e6 / BF16_PEAK_TF}
    out["split_planes_us"] = chain_us(split, dev)
    if graphs > 0:
        ref = state(lambda: drawcall(FORM_BY_SHAPE))
        out["draw_identical"] = all(bool(torch.equal(a, b)) for a, b in zip(ref, state(lambda: direct(graphs))))
        zt = chain_us(lambda: deg.zero_(), dev)
        for label, fn in (("draw_by_shape", lambda: drawcall(FORM_BY_SHAPE)), ("draw_form10", lambda: direct(graphs))):
            def f2(fn=fn):
                fn()
                deg.zero_()
            t = chain_us(f2, dev) - zt
            out[label] = {"chain_us": t, "bf16_frac": flop / t / 1e6 / BF16_PEAK_TF}
    print(json.dumps(out), flush=True)


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    if which in ("cora", "all"):
        run("cora-S1", 2708, 264, 6)
        run("citeseer-S1", 3327, 264, 6)
    if which in ("s16", "all"):
        run("cora-S16", 2708, 4224, 0)
        run("citeseer-S16", 3327, 4224, 0)
    if which == "graphs":  # the draw's cost per graph count (graph 0 only: the split prefetch)
        for gr in (1, 2, 6):
            run(f"cora-S1-g{gr}", 2708, 264, gr)
    if which in ("c5", "all"):
        run("synthetic20k-S1", 20000, 264, 6)


if __name__ == "__main__":
    main()
