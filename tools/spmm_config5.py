"""CSR-SpMM at BASELINE config 5 (synthetic N = 20 000, F = 16, dense θ ~ U(0,1)):
sample one graph with the product sampler, then time the aggregation kernels
(lds_spmm_norm: 16-lane row groups; lds_spmm_norm_blocked: column blocks of
s⊙Z in LDS; lds_aggregate_bitmask: the sampled bitmask × fixed-point s⊙Z on
the int8 matrix cores) with HIP events and check them against each other and against an
fp64 restatement on sampled rows.  Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "lds-gnn_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402

import ldsgnn  # noqa: E402
from ldsgnn import _native as nat  # noqa: E402
from ldsgnn.rng import TAG_GRAPH, tag_for  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "tools", "variants"))
import variants  # noqa: E402  (the tools-only variants library)

HBM_PEAK_GBS = 8000.0


def sample_csr(theta, n, seed=20000):
    dev = theta.device
    words = nat.lib.lds_bitmask_words(n)
    bits = torch.empty((n, words), dtype=torch.int64, device=dev)
    deg = torch.empty(n, dtype=torch.int32, device=dev)
    s = torch.empty(n, dtype=torch.float32, device=dev)
    rp = torch.empty(n + 1, dtype=torch.int32, device=dev)
    st = nat.stream_of(dev)
    nat.call("lds_sample_bitmask", nat.ptr(theta), n, seed, tag_for(TAG_GRAPH, 0), 0, 0, nat.ptr(bits), words, st)
    nat.call("lds_bitmask_degree", nat.ptr(bits), n, words, nat.ptr(deg), nat.ptr(s), st)
    nat.call("lds_exclusive_scan", nat.ptr(deg), n, nat.ptr(rp), st)
    nnz = int(rp[n].item())
    col = torch.empty(nnz, dtype=torch.int32, device=dev)
    nat.call("lds_bitmask_fill_csr", nat.ptr(bits), n, words, nat.ptr(rp), nat.ptr(col), nnz, 0, st)
    return rp, col, s, nnz, bits, words


def time_it(fn, reps):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return 1000.0 * a.elapsed_time(b) / reps  # µs


def main(n=20000, f=16, reps=20, high=1.0):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(20000)
    theta = torch.rand(n * (n + 1) // 2, generator=g, device=dev) * high
    rp, col, s, nnz, bits, words = sample_csr(theta, n)
    del theta
    z = torch.randn((n, f), generator=g, device=dev)
    st = nat.stream_of(dev)
    y_row = torch.empty((n, f), device=dev)
    y_blk = torch.empty((n, f), device=dev)
    nb = nat.lib.lds_spmm_block_count(n)
    bptr = torch.empty(n * (nb + 1), dtype=torch.int32, device=dev)
    part = torch.empty((nb, n, 16), device=dev)
    nat.call("lds_csr_block_ptr", nat.ptr(rp), nat.ptr(col), n, nat.ptr(bptr), st)

    def row():
        nat.call("lds_spmm_norm", nat.ptr(rp), nat.ptr(col), nat.ptr(s), n, nat.ptr(z), f, f, nat.ptr(y_row), f, 0, st)

    def blk():
        nat.call("lds_spmm_norm_blocked", nat.ptr(bptr), nat.ptr(col), nat.ptr(s), n, nat.ptr(z), f,
                 nat.ptr(y_blk), f, 0, nat.ptr(part), st)

    y_bit = torch.empty((n, f), device=dev)
    ws = torch.empty(int(nat.lib.lds_bitmask_agg_ws_bytes(n)), dtype=torch.uint8, device=dev)

    def bit():
        nat.call("lds_aggregate_bitmask", nat.ptr(bits), words, nat.ptr(s), n, nat.ptr(z), f, nat.ptr(y_bit), f, 0,
                 nat.ptr(ws), st)

    y_dn = torch.empty((n, f), device=dev)
    ws_dn = torch.empty(variants.ws_bytes(n), dtype=torch.uint8, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)

    def dense(quantize=1, grid=0, checked=True):
        nat.call("lds_spmm_norm_dense", nat.ptr(rp), nat.ptr(col), nat.ptr(s), n, nat.ptr(z), f, nat.ptr(y_dn), f, 0,
                 nat.ptr(ws_dn), grid, quantize, nat.ptr(err) if checked else 0, st)

    t_bp = time_it(lambda: nat.call("lds_csr_block_ptr", nat.ptr(rp), nat.ptr(col), n, nat.ptr(bptr), st), 3)
    t_row = time_it(row, reps)
    t_blk = time_it(blk, reps)
    t_bit = time_it(bit, reps)
    t_dn = time_it(dense, reps)  # (the digits of this s, z are in ws from here on)
    y_main = y_dn.clone()
    t_tile = time_it(lambda: dense(0, -256), reps)  # round 3's tile kernel (product only)
    y_abl0 = torch.empty_like(y_dn)
    eq_variants = {}
    for dbg in (20, 21, 22, 23, 33, 34, 6, 36, 37, 38, 39, 41, 42, 43, 44, 45, 46, 47, 48, 49, 50, 51, 52, 53, 54, 55, 56, 57, 60, 61, 62, 63, 64, 65, 66, 67, 68, 69):  # the product variants give the same bits
        variants.spmm_dense(nat.ptr(rp), nat.ptr(col), nat.ptr(s), n, nat.ptr(z), f, nat.ptr(y_abl0), f,
                            nat.ptr(ws_dn), dbg, st)
        eq_variants[dbg] = bool(torch.equal(y_abl0, y_main))
    y_tile = y_dn.clone()
    t_dn_main = time_it(lambda: dense(0), reps)
    # the unchecked form (err = NULL: the caller vouches for canonical columns,
    # as the engine and SampledGraph do): the call and the product
    t_dn_u = time_it(lambda: dense(1, 0, False), reps)
    t_dn_main_u = time_it(lambda: dense(0, 0, False), reps)
    eq_unchecked = bool(torch.equal(y_dn, y_main))
    y_abl = torch.empty_like(y_dn)
    abl = {}
    quick = bool(os.environ.get("SPMM5_QUICK"))  # product timings only, no ablations
    only = {int(c) for c in os.environ.get("SPMM5_ABL", "").split(",") if c}  # time just these codes
    for dbg, what in () if quick and not only else ((6, "row-block kernel, digits by register loads, bits by LDS-DMA (product)"),
                      (7, "row-block: hybrid multiply phase alone"),
                      (8, "row-block: hybrid multiply phase alone, no per-chunk barrier"),
                      (23, "spill-pass kernel, ring depth 8"), (36, "spill-pass, quad-reduced bit setting"),
                      (37, "spill-pass, windowed bit setting on every step"),
                      (38, "spill-pass, windowed bit setting, ring depth 6"),
                      (39, "spill-pass, ring read one step ahead of the bit ORs"),
                      (40, "spill-pass, interior ORs as plain stores (timing only)"),
                      (41, "spill-pass, ring loop not unrolled"), (42, "spill-pass, ring loop not unrolled, depth 12"),
                      (43, "spill-pass, 12 streaming + 4 multiply waves, depth 5"),
                      (44, "spill-pass, 12 streaming + 4 multiply waves, depth 6"),
                      (45, "spill-pass, 12 streaming waves, depth 4"), (47, "spill-pass, 12 streaming waves, depth 3"),
                      (46, "spill-pass, 12 streaming waves, depth 5, windowed boundary steps"),
                      (48, "spill-pass, 14 streaming + 2 multiply waves, depth 4"), (49, "spill-pass, 14 streaming waves, depth 3"),
                      (50, "spill-pass, 12 streaming waves, depth 4, fast path for spills"),
                      (51, "spill-pass, 14 streaming waves, depth 4, fast path for spills"),
                      (52, "spill-pass, 12 streaming waves, depth 4, fast paths for spills and boundary lanes"),
                      (53, "spill-pass, 12 streaming waves, depth 3, fast paths for spills and boundary lanes"),
                      (54, "spill-pass, 12 streaming waves, 2-KB steps, depth 3, fast paths"),
                      (55, "spill-pass, 12 streaming waves, 2-KB steps, LDS ring depth 2, fast paths"),
                      (56, "spill-pass, 8 streaming waves, 2-KB steps, depth 2, fast paths"),
                      (57, "spill-pass, 14 streaming waves, 2-KB steps, depth 2, fast paths"),
                      (58, "spill-pass, 2-KB steps, LDS ring depth 2, without bit setting (timing only)"),
                      (59, "spill-pass, 2-KB steps, LDS ring depth 2, without MFMAs (timing only)"),
                      (60, "spill-pass, register ring depth 3"), (61, "spill-pass, register ring depth 4"),
                      (62, "spill-pass, register ring depth 6"),
                      (63, "spill-pass, register ring depth 4, rows taken per pass from a counter"),
                      (64, "spill-pass, register ring depth 4, per-(row, pass) constants cached (the product form)"),
                      (65, "spill-pass, product form with lean fast-path ORs and one wave-wide skip"),
                      (66, "spill-pass, product form with one ballot for the step flags"),
                      (67, "spill-pass, product form with 14 streaming + 2 multiply waves"),
                      (68, "spill-pass, product form with 3-KB steps, depth 3"), (69, "spill-pass, product form with 3-KB steps, depth 4"),
                      (33, "spill-pass, ring depth 6"),
                      (34, "spill-pass, ring depth 12"), (31, "spill-pass, no MFMAs"),
                      (32, "spill-pass, streaming without bit setting"),
                      (20, "column-pass, 8 streaming + 8 multiply waves"),
                      (21, "column-pass, 16 waves streaming then multiplying"),
                      (22, "row-block kernel, multiply phase staged by LDS-DMA"),
                      (11, "column-pass concurrent, no multiply"), (12, "column-pass concurrent, no streaming"),
                      (13, "column-pass sequential, no multiply"),
                      (1, "row-block: streaming phase alone"), (2, "row-block: streaming without bit-row stores"),
                      (3, "row-block: multiply phase alone"), (4, "row-block: multiply without bit-row loads"),
                      (5, "row-block: streaming without stores + column-pass step bookkeeping")):
        if only and dbg not in only:
            continue
        abl[what] = time_it(lambda: variants.spmm_dense(nat.ptr(rp), nat.ptr(col), nat.ptr(s), n,
                                                        nat.ptr(z), f, nat.ptr(y_abl), f, nat.ptr(ws_dn), dbg, st), reps)
    dense(0)  # the product again (the multiply-only ablation left its slabs in place)
    # parity: blocked vs row kernel (fp32, different order) and fp64 on sampled rows
    rel = float((y_blk - y_row).abs().max() / y_row.abs().max())
    rows = torch.randint(0, n, (32,), generator=g, device=dev)
    err64 = err64_bit = 0.0
    for i in rows.tolist():
        js = col[rp[i]:rp[i + 1]].long()
        ref = (s[i].double() * (s[js].double()[:, None] * z[js].double()).sum(0))
        err64 = max(err64, float((y_blk[i].double() - ref).abs().max() / ref.abs().max()))
        err64_bit = max(err64_bit, float((y_bit[i].double() - ref).abs().max() / ref.abs().max()))
    # bitmask path: the mask (n rows × words uint64), s, Z in, Y out
    algo_bit = 8 * n * words + 4 * n + 8 * n * f
    algo = 4 * (n + 1) + 4 * nnz + 4 * n + 8 * n * f
    out = {"workload": f"config5 synthetic N={n} F={f} theta~U(0,{high})", "nnz": nnz,
           "algorithmic_bytes": algo,
           "row_kernel": {"avg_us": t_row, "achieved_GBs": algo / t_row / 1e3, "frac": algo / t_row / 1e3 / HBM_PEAK_GBS},
           "blocked_kernel": {"avg_us": t_blk, "achieved_GBs": algo / t_blk / 1e3,
                              "frac": algo / t_blk / 1e3 / HBM_PEAK_GBS, "block_ptr_us": t_bp},
           "bitmask_kernel": {"avg_us": t_bit, "algorithmic_bytes": algo_bit, "achieved_GBs": algo_bit / t_bit / 1e3,
                              "frac": algo_bit / t_bit / 1e3 / HBM_PEAK_GBS,
                              "speedup_vs_blocked": t_blk / t_bit},
           "dense_csr_kernel": {"avg_us_call": t_dn, "achieved_GBs_call": algo / t_dn / 1e3,
                                "frac_call": algo / t_dn / 1e3 / HBM_PEAK_GBS, "avg_us_product": t_dn_main,
                                "achieved_GBs_product": algo / t_dn_main / 1e3,
                                "frac_product": algo / t_dn_main / 1e3 / HBM_PEAK_GBS,
                                "unchecked": {"avg_us_call": t_dn_u, "frac_call": algo / t_dn_u / 1e3 / HBM_PEAK_GBS,
                                              "avg_us_product": t_dn_main_u,
                                              "frac_product": algo / t_dn_main_u / 1e3 / HBM_PEAK_GBS,
                                              "equal_to_checked": eq_unchecked},
                                "speedup_vs_blocked": t_blk / t_dn,
                                "max_rel_vs_row": float((y_dn - y_row).abs().max() / y_row.abs().max()),
                                "tile_kernel_us_product": t_tile,
                                "tile_kernel_frac_product": algo / t_tile / 1e3 / HBM_PEAK_GBS,
                                "equal_to_tile_kernel": bool(torch.equal(y_main, y_tile)),
                                "ablations_us": abl, "variants_equal": eq_variants,
                                "equal_to_bitmask": bool(torch.equal(y_dn, y_bit)),
                                "error_word": int(err.item())},
           "max_rel_blocked_vs_row": rel, "max_rel_vs_fp64_rows": err64,
           "max_rel_bitmask_vs_row": float((y_bit - y_row).abs().max() / y_row.abs().max()),
           "max_rel_bitmask_vs_fp64_rows": err64_bit}
    print(json.dumps(out))


if __name__ == "__main__":
    main(high=float(sys.argv[1]) if len(sys.argv) > 1 else 1.0)
