"""Is the W0-products launch (lds_engine_xt_adam) bound by its fused final
reduction block?  The C-ABI calls of one eager Cora window are recorded (as
bench.py's window breakdown does); each xt_adam call is chain-timed as
recorded and with the final reduction dropped (partials = NULL)."""
import json
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lds-gnn_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


def main():
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
    out = []
    for i, (name, a) in enumerate(c for c in calls if c[0] == "lds_engine_xt_adam"):
        full = bench.chain_us(lambda st, a=a: real(name, *(a[:-1] + (st,))), dev, 20)
        a2 = a[:14] + (0,) + a[15:]
        nofin = bench.chain_us(lambda st, a2=a2: real(name, *(a2[:-1] + (st,))), dev, 20)
        out.append({"call": i, "us": full, "us_without_final_block": nofin, "nblocks": a[15]})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
