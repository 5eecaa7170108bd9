"""What the in-tile degree count costs the window sampler (run under
rocprofv3 --kernel-trace --stats): the bench workload's recorded window draw
replayed 50 times as recorded (tiles count degrees with atomics, then the fused
fill), then 50 times without CSR (col = NULL: the tile kernel without degree
atomics, then degree_kernel).  Compare sample_tiles_kernel<false, true, true>
against <false, true, false> in the kernel stats.
usage: python tools/diag/sampler_deg_ab.py"""
import argparse
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "lds-gnn_amd")]

import torch  # noqa: E402


def main():
    import bench
    from ldsgnn import _native as nat
    bargs = argparse.Namespace(dataset="cora", seed=597905255 % (2 ** 31), samples=1, graph_model="lds")
    dev = torch.device("cuda", 0)
    _, runner, _ = bench.build(bargs, 0, dev)
    eng, _ = bench.make_engine(runner, 5, 1, 1)
    eng.inner_step()
    eng.hyper_step()
    calls = []
    real = nat.call

    def rec(name, *a):
        calls.append((name, a))
        real(name, *a)

    nat.call = rec
    eng.run_window(5)
    nat.call = real
    torch.cuda.synchronize()
    draw = [a for name, a in calls if name == "lds_sample_graphs_multi"][0]
    fused = draw[:-3] + (0,) + draw[-2:]          # clears its own workspace
    bits_only = fused[:13] + (None,) + fused[14:]  # col = NULL
    for label, a in (("fused", fused), ("bits_only", bits_only)):
        for _ in range(50):
            real("lds_sample_graphs_multi", *a)
        torch.cuda.synchronize()
        print(label, "done", flush=True)


if __name__ == "__main__":
    main()
