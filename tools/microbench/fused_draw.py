"""θ-grad + SGD with the next window's draw fused into its epilogue
(lds_theta_grad_sgd_draw) against the separate θ-grad + SGD and batched draw
(lds_theta_grad_sgd, then lds_sample_graphs_multi with CSR), at the Cora
window shape (n 2708, k 264, 6 graphs).  Each path runs as a dependent chain
of 20 copies from one HIP graph, timed with HIP events; per-kernel averages
come from running it under rocprofv3 --kernel-trace --stats."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lds-gnn_amd")]
import torch  # noqa: E402

import ldsgnn  # noqa: E402,F401
from ldsgnn import _native as nat  # noqa: E402
from ldsgnn.rng import TAG_GRAPH, tag_for  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    n, k, graphs = 2708, 264, 6
    g = torch.Generator(device=dev).manual_seed(1)
    u = torch.randn((n, k), generator=g, device=dev) * 0.01
    v = torch.randn((n, k), generator=g, device=dev) * 0.01
    r = torch.randn(n, generator=g, device=dev) * 0.01
    theta = torch.rand(n * (n + 1) // 2, generator=g, device=dev) * 0.02
    scal = torch.zeros(64, dtype=torch.uint8, device=dev)
    scal[16:24].view(torch.float64).fill_(1e-6)
    st = nat.stream_of(dev)
    words = nat.lib.lds_bitmask_words(n)
    wsi = nat.lib.lds_sample_ws_ints(n)
    base = torch.zeros(4, dtype=torch.int32, device=dev)
    bits = torch.zeros((graphs, n, words), dtype=torch.int64, device=dev)
    deg = torch.zeros((graphs, wsi), dtype=torch.int32, device=dev)
    cap = 200_000
    row_ptr = torch.zeros((graphs, n + 1), dtype=torch.int32, device=dev)
    col = torch.zeros((graphs, cap), dtype=torch.int32, device=dev)
    s = torch.zeros((graphs, n), dtype=torch.float32, device=dev)
    ell = torch.zeros((graphs, n, 64, 2), dtype=torch.int32, device=dev)
    seed, tag = 99, tag_for(TAG_GRAPH, 0)

    def separate():
        nat.call("lds_theta_grad_sgd", nat.ptr(u), nat.ptr(v), k, k, nat.ptr(r), 1, 1, nat.ptr(theta), n, 0,
                 nat.ptr(scal), 1, nat.stream_of(dev))
        nat.call("lds_sample_graphs_multi", nat.ptr(theta), n, seed, tag, 1, nat.ptr(base), 0, graphs, 1,
                 nat.ptr(bits), words, nat.ptr(deg), nat.ptr(row_ptr), nat.ptr(col), cap, nat.ptr(s), nat.ptr(ell),
                 0, 0, 0, nat.stream_of(dev))

    def fused():
        nat.call("lds_theta_grad_sgd_draw", nat.ptr(u), nat.ptr(v), k, k, nat.ptr(r), 1, 1, nat.ptr(theta), n, 0,
                 nat.ptr(scal), seed, tag, nat.ptr(base), 0, graphs, nat.ptr(bits), words, nat.ptr(deg), 1,
                 nat.stream_of(dev))
        deg.zero_()  # the engine would clear it elsewhere; keeps the atomics bounded here

    def plain():
        nat.call("lds_theta_grad_sgd", nat.ptr(u), nat.ptr(v), k, k, nat.ptr(r), 1, 1, nat.ptr(theta), n, 0,
                 nat.ptr(scal), 1, nat.stream_of(dev))

    out = {"n": n, "k": k, "graphs": graphs}
    for name, fn in (("separate", separate), ("fused", fused), ("plain_theta_grad", plain)):
        fn()
        torch.cuda.synchronize()
        s_ = torch.cuda.Stream(dev)
        s_.wait_stream(torch.cuda.current_stream(dev))
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s_):
            with torch.cuda.graph(graph, stream=s_):
                for _ in range(20):
                    fn()
        torch.cuda.current_stream(dev).wait_stream(s_)
        graph.replay()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            graph.replay()
        b.record()
        torch.cuda.synchronize()
        out[name + "_us"] = 1000.0 * a.elapsed_time(b) / 200
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
