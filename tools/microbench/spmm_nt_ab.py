"""A/B of the config-5 CSR-SpMM's column stream cache policy (round 6): the
product spill-pass kernel (default policy) against the same kernel with
`global_load_dwordx4 … nt` on the stream, interleaved over three rounds,
checked and unchecked, after one quantising product call; equal results
required.  One JSON line on stdout."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lds-gnn_amd"), os.path.join(ROOT, "tools"),
                os.path.join(ROOT, "tools", "variants")]
import torch  # noqa: E402

from ldsgnn import _native as nat  # noqa: E402
import variants  # noqa: E402
from spmm_config5 import sample_csr, time_it  # noqa: E402

HBM = 8000.0


def main(n=20000, f=16, reps=20, rounds=3):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(20000)
    theta = torch.rand(n * (n + 1) // 2, generator=g, device=dev)
    rp, col, s, nnz, bits, words = sample_csr(theta, n)
    del theta, bits
    z = torch.randn((n, f), generator=g, device=dev)
    st = nat.stream_of(dev)
    ws = torch.empty(variants.ws_bytes(n), dtype=torch.uint8, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    y0, y1 = torch.empty((n, f), device=dev), torch.empty((n, f), device=dev)
    P = nat.ptr

    def prod(quantize=0, checked=False):
        nat.call("lds_spmm_norm_dense", P(rp), P(col), P(s), n, P(z), f, P(y0), f, 0, P(ws), 0, quantize,
                 P(err) if checked else 0, st)

    def nt(checked=False):
        variants.spmm_dense_nt(P(rp), P(col), P(s), n, P(y1), f, P(ws), 0, P(err) if checked else 0, st)

    prod(1)
    torch.cuda.synchronize()
    algo = 4 * (n + 1) + 4 * nnz + 4 * n + 8 * n * f
    res = {"workload": f"config5 n={n}", "nnz": nnz, "algorithmic_bytes": algo, "rounds": []}
    for _ in range(rounds):
        res["rounds"].append({"product_us": time_it(lambda: prod(), reps), "nt_us": time_it(lambda: nt(), reps),
                              "product_checked_us": time_it(lambda: prod(checked=True), reps),
                              "nt_checked_us": time_it(lambda: nt(True), reps)})
    nt()
    prod()
    torch.cuda.synchronize()
    res["equal"] = bool(torch.equal(y0, y1))
    res["error_word"] = int(err.item())
    best = {k: min(r[k] for r in res["rounds"]) for k in res["rounds"][0]}
    res["best_us"] = best
    res["best_frac"] = {k: algo / v / 1e3 / HBM for k, v in best.items()}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
