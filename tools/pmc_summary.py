"""Per-kernel HBM traffic from the two rocprofv3 PMC passes of tools/gpu.sh (pmc, pmc5).

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE counts
half the bytes of a wide coalesced read (MI355X_MICROARCH.md, HBM section), so
the read bytes are reported as 2 x FETCH_SIZE; WRITE_SIZE is taken as is.
Usage: python tools/pmc_summary.py gpurun_out/pmc_<tag> [kernel-substring] [--json out.json]
"""
import csv
import json
import sys
from collections import defaultdict


def load(path):
    per = defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            per[row["Kernel_Name"].split("(")[0]].append(float(row["Counter_Value"]))
    return per


# engine entry point -> the kernels one call of it dispatches (name substrings)
ENTRY_KERNELS = {
    # the window's batched draw: graphs looped in the tile kernel (kLoop, kDeg) + the fused fill
    # (the single-graph <false, false, true> draws of the step-0 window are not this entry's launches)
    "lds_sample_graphs_multi": ["lds::sample_tiles_kernel<false, true, true>", "lds::fill_csr_fused_kernel"],
    "lds_sample_fill_csr": ["lds::fill_csr_fused_kernel", "lds::degree_scale_kernel"],
    # θ-grad + SGD; with the next window's draw fused in: the DRAW = true instance
    "lds_theta_grad_sgd": ["theta_grad_bf3_kernel<16, true, false, true, false>", "theta_grad_bf3_t128",
                           "theta_grad_bf3_pipe", "theta_grad_mfma", "theta_grad_w8_kernel<true, false, false>",
                           "theta_grad_w8_kernel<false, false, false>"],
    "lds_theta_grad_direct": ["theta_grad_dma_kernel"],
    "lds_theta_grad_sgd_draw": ["theta_grad_bf3_kernel<16, true, false, true, true>",
                                "theta_grad_w8_kernel<true, false, true>", "theta_grad_w8_kernel<false, false, true>",
                                "theta_grad_bf3_t128_kernel<true, true, false, true>",
                                "theta_grad_bf3_t128_kernel<true, false, false, true>"],
    "lds_engine_x_linear": ["lds::x_linear_kernel"],
    "lds_engine_fill_x_linear": ["fill_x_linear_kernel"],
    "lds_engine_fwd_layer1": ["fwd_layer1_kernel"],
    "lds_engine_fwd_layer2": ["fwd_layer2_kernel"],
    "lds_engine_bwd_layer2": ["bwd_layer2_kernel"],
    "lds_engine_fwd2_bwd2": ["fwd2_bwd2_kernel"],
    "lds_engine_rev_bc": ["rev_bc_kernel"],
    "lds_engine_bwd1_reduce": ["bwd1_reduce_kernel"],
    "lds_engine_xt_adam": ["xt_adam_kernel"],
    "lds_engine_rev_a": ["rev_a_kernel"],
    "lds_engine_rev_b": ["rev_b_kernel"],
    "lds_engine_rev_c": ["rev_c_kernel"],
    "lds_engine_rev_d_reduce": ["rev_d_reduce_kernel"],
    "lds_engine_end_window": ["end_window_kernel"],
    # config 5 (long rows, bitmask aggregation): the aggregation's prepasses and product, the split W0 products
    "lds_aggregate_bitmask_partials": ["bitagg_colmax_kernel", "bitagg_quant_kernel", "bitagg_main_kernel"],
    "lds_engine_xt_partials": ["xt_partials_kernel"],
}


def entries(per_kernel):
    """Bytes per call of each entry point: the sum over its kernels of their
    per-dispatch means."""
    out = {}
    for entry, subs in ENTRY_KERNELS.items():
        ks = [k for k in per_kernel if any(s in k for s in subs)]
        if not ks:
            continue
        out[entry] = {f: sum(per_kernel[k][f] for k in ks) for f in ("read_bytes", "write_bytes", "traffic_bytes")}
        out[entry]["kernels"] = ks
    return out


def main():
    base = sys.argv[1]
    want = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else None
    fetch = load(f"{base}_fetch/run_counter_collection.csv")
    write = load(f"{base}_write/run_counter_collection.csv")
    out = {}
    for name in sorted(set(fetch) | set(write), key=lambda k: -sum(fetch.get(k, [0]))):
        if want and want not in name:
            continue
        f, w = fetch.get(name, []), write.get(name, [])
        if not f or not w:
            continue
        rd = 2 * 1024 * sum(f) / len(f)
        wr = 1024 * sum(w) / len(w)
        out[name] = dict(launches=len(f), read_bytes=rd, write_bytes=wr, traffic_bytes=rd + wr)
        print(f"{len(f):6d} read {rd / 1e6:9.3f} MB  write {wr / 1e6:9.3f} MB  per launch  {name}")
    ent = entries(out)
    for name, e in ent.items():
        print(f"entry {name}: read {e['read_bytes'] / 1e6:.3f} MB write {e['write_bytes'] / 1e6:.3f} MB per call")
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as fh:
            json.dump({**ent, "_kernels": out}, fh, indent=1)


if __name__ == "__main__":
    main()
