"""θ-grad + SGD + next-window draw (lds_theta_grad_sgd_draw): the 64-tile form
(form 6) against the eight-wave 128-tile form (form 9), and the plain θ-grad
+ SGD (lds_theta_grad_ex mode 2) of the forms named in THETA_FORMS, at the
engine's shapes.  Checks that the two draw forms give identical θ, bit rows and
degree counts, then times each as a dependent chain of 20 copies in one HIP
graph (HIP events on the launch stream).  One JSON line per shape.
Usage (GPU box): python tools/microbench/tg_draw_ab.py [cora|c5|all]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lds-gnn_amd")]
import torch  # noqa: E402

import ldsgnn  # noqa: E402,F401
from ldsgnn import _native as nat  # noqa: E402
from ldsgnn import ops  # noqa: E402
from ldsgnn.rng import TAG_GRAPH, tag_for  # noqa: E402

BF16_PEAK_TF = 2500.0
# draw forms compared (the first is the reference for the bit-identity check)
DRAW_FORMS = tuple(os.environ.get("DRAW_FORMS", "bf16x3-t64k16-grouped,bf16x3-t128-w8").split(","))


def chain_us(fn, dev, copies=20, reps=10):
    fn()
    torch.cuda.synchronize()
    s_ = torch.cuda.Stream(dev)
    s_.wait_stream(torch.cuda.current_stream(dev))
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s_):
        with torch.cuda.graph(graph, stream=s_):
            for _ in range(copies):
                fn()
    torch.cuda.current_stream(dev).wait_stream(s_)
    graph.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        graph.replay()
    b.record()
    torch.cuda.synchronize()
    return 1000.0 * a.elapsed_time(b) / (copies * reps)


def run(name, n, k, graphs, plain_forms):
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
    seed, tag = 99, tag_for(TAG_GRAPH, 0)
    flop = 24.0 * k * n * (n + 1) / 2  # bf16 MFMA flop (six products per fp32 product)
    out = {"workload": name, "n": n, "k": k, "graphs": graphs}

    def draw_call():
        nat.call("lds_theta_grad_sgd_draw", nat.ptr(u), nat.ptr(v), k, k, nat.ptr(r), 1, 1, nat.ptr(theta), n,
                 nat.ptr(grad), nat.ptr(scal), seed, tag, nat.ptr(base), 0, graphs, nat.ptr(bits), words,
                 nat.ptr(deg), ops.form_code(), nat.stream_of(dev))

    results = {}
    for form in DRAW_FORMS:
        prev = ops.theta_grad_form(form)
        try:
            theta.copy_(theta0)
            bits.zero_()
            deg.zero_()
            draw_call()
            torch.cuda.synchronize()
            results[form] = (theta.clone(), grad.clone(), bits.clone(), deg.clone())

            def fn():
                draw_call()
                deg.zero_()  # keeps the degree atomics bounded; its own chain time is subtracted
            t = chain_us(fn, dev)
            zt = chain_us(lambda: deg.zero_(), dev)
            out["draw_" + form] = {"chain_us": t - zt, "bf16_frac": flop / (t - zt) / 1e6 / BF16_PEAK_TF}
        finally:
            ops.theta_grad_form(prev)
    a = results[DRAW_FORMS[0]]
    out["draw_identical"] = {f: all(bool(torch.equal(x, y)) for x, y in zip(a, results[f])) for f in DRAW_FORMS[1:]}
    for form in plain_forms:
        prev = ops.theta_grad_form(form)
        try:
            def fn():
                nat.call("lds_theta_grad_ex", nat.ptr(u), nat.ptr(v), k, k, nat.ptr(r), 1, n, 1, nat.ptr(theta), n,
                         nat.ptr(grad), 2, nat.ptr(scal), 1.0, ops.form_code(), nat.stream_of(dev))
            theta.copy_(theta0)
            fn()
            torch.cuda.synchronize()
            same = bool(torch.equal(grad, results["bf16x3-t64k16-grouped"][1]))
            t = chain_us(fn, dev)
            out["plain_" + form] = {"chain_us": t, "bf16_frac": flop / t / 1e6 / BF16_PEAK_TF, "grad_equal": same}
        finally:
            ops.theta_grad_form(prev)
    print(json.dumps(out), flush=True)


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    forms = tuple(os.environ.get("THETA_FORMS", "bf16x3-t64k16-grouped,bf16x3-t128-grouped,bf16x3-t128-pipe,"
                                 "bf16x3-t128-w8").split(","))
    if which in ("cora", "all"):
        run("cora-S1", 2708, 264, 6, forms)
        run("citeseer-S1", 3327, 264, 6, forms)
    if which in ("s16", "all"):
        run("cora-S16", 2708, 4224, 1, forms)
        run("citeseer-S16", 3327, 4224, 1, forms)
    if which in ("c5", "all"):
        run("synthetic20k-S1", 20000, 264, 6, forms)


if __name__ == "__main__":
    main()
