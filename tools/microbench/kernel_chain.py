"""Where a τ-window's time goes, launch by launch.

Records the C-ABI calls of one eager engine window (bench.py's default
workload), then for every recorded call replays K back-to-back copies of it
from one HIP graph (a dependent chain of that launch alone) and reports the
per-launch time, next to a trivial-kernel floor and the replayed window.
Outputs one JSON line per call plus a summary line.

usage: python tools/microbench/kernel_chain.py [--samples S] [--dataset cora]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "lds-gnn_amd")]

import torch  # noqa: E402


def graph_time(fn, reps=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=1)
    ap.add_argument("--dataset", default="cora")
    ap.add_argument("--k", type=int, default=100)
    args = ap.parse_args()
    import bench
    from ldsgnn import _native as nat
    bargs = argparse.Namespace(dataset=args.dataset, seed=597905255 % (2 ** 31), samples=args.samples,
                               graph_model="lds")
    dev = torch.device("cuda", 0)
    data, runner, _ = bench.build(bargs, 0, dev)
    eng, _ = bench.make_engine(runner, 5, 1, args.samples)
    eng.inner_step()
    eng.hyper_step()
    eng.run_window(5)
    torch.cuda.synchronize()

    calls = []
    real = nat.call

    def rec(name, *a):
        calls.append((name, a))
        real(name, *a)

    nat.call = rec
    eng.run_window(5)
    nat.call = real
    torch.cuda.synchronize()

    def cur(a):  # every entry point takes its stream last: launch on the capturing stream
        return a[:-1] + (nat.stream_of(dev),)

    def replay_all():
        for name, a in calls:
            real(name, *cur(a))

    t_window = graph_time(replay_all)
    scal = torch.zeros(32, dtype=torch.uint8, device=dev)
    floor = graph_time(lambda: [real("lds_engine_advance", nat.ptr(scal), 0, 0, 0, 0, nat.stream_of(dev))
                                for _ in range(args.k)])
    print(json.dumps({"what": "floor", "kernel": "lds_engine_advance (1 block)", "us": 1e6 * floor / args.k}))
    rows = []
    ws_bytes = eng.gbatch.deg.numel() * 4
    memset = graph_time(lambda: [torch.cuda.current_stream() and eng.gbatch.deg.zero_() for _ in range(args.k)])
    print(json.dumps({"what": "memset chain", "bytes": ws_bytes, "us": 1e6 * memset / args.k}), flush=True)
    for i, (name, a) in enumerate(calls):
        if name == "lds_sample_graphs_multi":  # repeated draws: the call clears its workspace (ws_zeroed = 0)
            a = a[:-3] + (0,) + a[-2:]

        def chain(name=name, a=a):
            for _ in range(args.k):
                real(name, *cur(a))
        t = graph_time(chain) / args.k
        rows.append({"i": i, "call": name, "us": 1e6 * t})
        print(json.dumps(rows[-1]), flush=True)
    # ablations of the W0-product launch: without the fused final reduction
    # block, without the heavy-column blocks (every column one wave)
    xt = [a for name, a in calls if name == "lds_engine_xt_adam"]
    if xt:
        a = xt[0]
        for label, b in (("as recorded", a), ("no final block", a[:14] + (0,) + a[15:]),
                         ("no heavy columns, no heads", a[:-5] + (0, 0, 0) + a[-2:])):
            def chain(b=b):
                for _ in range(args.k):
                    real("lds_engine_xt_adam", *cur(b))
            print(json.dumps({"what": "xt_adam ablation", "variant": label, "us": 1e6 * graph_time(chain) / args.k}),
                  flush=True)
    # two-hop kernels without picks (mask bit no node has): the walk + epilogue alone
    for name in ("lds_engine_fwd2_bwd2", "lds_engine_rev_bc"):
        for i, a in enumerate([a for nm, a in calls if nm == name][:1] + [a for nm, a in calls if nm == name][-1:]):
            b = a[:6] + (128,) + a[7:]
            for label, x in (("as recorded", a), ("no picks", b)):
                def chain(x=x, name=name):
                    for _ in range(args.k):
                        real(name, *cur(x))
                print(json.dumps({"what": "two-hop ablation", "call": name, "which": "first" if i == 0 else "last",
                                  "variant": label, "us": 1e6 * graph_time(chain) / args.k}), flush=True)
    print(json.dumps({"what": "summary", "calls": len(calls), "window_us": 1e6 * t_window,
                      "sum_self_chain_us": sum(r["us"] for r in rows), "floor_us": 1e6 * floor / args.k,
                      "samples": args.samples}))


if __name__ == "__main__":
    main()
