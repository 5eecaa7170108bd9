"""Which part of the W0-products launch (lds_engine_xt_adam) sets its time at
Cora S = 1?  The C-ABI calls of one eager window are recorded (as
tools/microbench/xt_final.py does) and every xt_adam call is chain-timed
(20 dependent copies in one HIP graph).  Run once per library (LDSGNN_LIB):
the product, and timing-only builds of engine.hip with -DLDS_XT_EXPT=k
(tools/variants/xt/lib_xtk.so): 1 heavy-column blocks exit at once, 2 the
one-column light waves exit, 3 the two- / four-column light waves exit,
4 the final-reduction blocks exit, 5 every block exits at entry (the grid's
launch floor), 6 no Adam (mode 0), 7 the Adam operands loaded after the
product, 8 no m / v / g' stores, 9 no Adam operand loads, 10 the operands
loaded but no update computed or stored — their results are wrong by
construction (profiles/r06_xt_parts.jsonl).
Usage (GPU box): LDSGNN_LIB=... python tools/microbench/xt_parts.py LABEL [ENTRY]
(ENTRY: another engine entry point of the window, e.g. lds_engine_x_linear)"""
import json
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lds-gnn_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    label = sys.argv[1] if len(sys.argv) > 1 else "product"
    entry = sys.argv[2] if len(sys.argv) > 2 else "lds_engine_xt_adam"  # any engine entry of the window
    dev = torch.device("cuda:0")
    args = types.SimpleNamespace(dataset="cora", seed=597905255 % (2 ** 31), samples=1, graph_model="lds",
                                 gae_dropout=0.0, tau=5)
    data, runner, _ = bench.build(args, 0, dev)
    eng, reducer = bench.make_engine(runner, 5, 1)
    eng.inner_step()
    eng.hyper_step()
    from ldsgnn import _native as nat
    calls, real = [], nat.call

    def rec(name, *a):
        calls.append((name, a))
        real(name, *a)
    nat.call = rec
    try:
        eng.run_window(5)
    finally:
        nat.call = real
    torch.cuda.synchronize()
    xt = [a for name, a in calls if name == entry]
    us = [min(bench.chain_us(lambda st, a=a: real(entry, *(a[:-1] + (st,))), dev, 20)
              for _ in range(3)) for a in xt]
    print(json.dumps({"lib": label, "entry": entry, "calls": len(us), "mean_us": round(sum(us) / len(us), 3),
                      "us": [round(u, 3) for u in us]}), flush=True)


if __name__ == "__main__":
    main()
