"""Per-rank compute of the band-sharded exchange at BASELINE config 5 and
N = 8, on one GPU: what one rank of eight runs per window
besides the collectives — the band θ-gradient over every rank's factors
(8 × K columns, 1/8 of the triangle, fused SGD + clamp), the band draws of
all eight replicas' six graphs, the packing of the band rows for the
all-to-all, the unpacking of the other bands, and the mirror + degree pass —
for the smallest, a middle and the largest band, next to what one GPU runs
now (the full-triangle assembly with its fused draw of six graphs).  Random
factors of the window's real width (K = 264 at τ = 5, C = 7).  One JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "lds-gnn_amd")]
import torch  # noqa: E402

from ldsgnn import _native as nat  # noqa: E402
from ldsgnn.replicas import band_bounds  # noqa: E402
from ldsgnn.rng import TAG_GRAPH, tag_for  # noqa: E402


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return 1000.0 * a.elapsed_time(b) / reps


def main(n=20000, K=264, N=8, count=6):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(7)
    st = nat.stream_of(dev)
    P = nat.ptr
    m = n * (n + 1) // 2
    theta = torch.rand(m, generator=g, device=dev)
    scal = torch.zeros(nat.lib.lds_engine_scalars_size(), dtype=torch.uint8, device=dev)
    scal[16:24].view(torch.float64).fill_(1e-12)  # (a tiny lr: θ stays ~U(0, 1) over the repeats)
    W = nat.lib.lds_bitmask_words(n)
    wsi = nat.lib.lds_sample_ws_ints(n)
    out = {"n": n, "K": K, "world": N, "graphs_per_replica": count}
    # one GPU now: the full assembly (K columns) with the six graphs' draw fused (the engine's config-5 launch)
    u1 = torch.randn((n, K), generator=g, device=dev) * 1e-3
    v1 = torch.randn((n, K), generator=g, device=dev) * 1e-3
    r1 = torch.randn((1, n), generator=g, device=dev) * 1e-3
    bits1 = torch.zeros((count, n, W), dtype=torch.int64, device=dev)
    deg1 = torch.zeros((count, wsi), dtype=torch.int32, device=dev)

    def full():
        deg1.zero_()
        nat.call("lds_theta_grad_sgd_draw", P(u1), P(v1), K, K, P(r1), 1, 1, P(theta), n, 0, P(scal), 99,
                 tag_for(TAG_GRAPH, 0), P(scal), 0, count, P(bits1), W, P(deg1), 1, st)
    out["one_gpu_theta_grad_draw_us"] = timed(full)
    # one rank of N: every rank's factors side by side
    uc = torch.randn((n, N * K), generator=g, device=dev) * 1e-3
    vc = torch.randn((n, N * K), generator=g, device=dev) * 1e-3
    rc = torch.randn((N, n), generator=g, device=dev) * 1e-3
    ab = torch.zeros((count, N, n, W), dtype=torch.int64, device=dev)
    bounds = band_bounds(n, N)
    bands = {}
    for b in (0, N // 2, N - 1):
        r0, r1_ = bounds[b]
        t_tg = timed(lambda: nat.call("lds_theta_grad_band", P(uc), P(vc), N * K, N * K, P(rc), 1, n, N, P(theta), n,
                                      0, 2, P(scal), 1.0 / N, r0, r1_, st))
        t_draw = timed(lambda: nat.call("lds_sample_band_bits", P(theta), n, 99, tag_for(TAG_GRAPH, 0), 1, P(scal), 0,
                                        count, N, r0, r1_, P(ab), W, st))
        t_pack = timed(lambda: ab[:, :, r0:r1_, r0 // 64:].permute(1, 0, 2, 3).contiguous())
        box = (r1_ - r0) * (W - r0 // 64)
        bands[b] = {"rows": [r0, r1_], "theta_grad_band_sgd_us": t_tg, "band_draw_all_replicas_us": t_draw,
                    "pack_us": t_pack, "sent_MB": count * (N - 1) * box * 8 / 1e6}
    out["bands"] = bands
    # the owner's side: unpack every band's rows into its six graphs, then mirror + degrees
    dst = torch.zeros((count, n, W), dtype=torch.int64, device=dev)
    recv = {q: torch.zeros((count, q1 - q0, W - q0 // 64), dtype=torch.int64, device=dev)
            for q, (q0, q1) in enumerate(bounds)}

    def unpack():
        for q, (q0, q1) in enumerate(bounds):
            dst[:, q0:q1, q0 // 64:] = recv[q]
    out["unpack_us"] = timed(unpack)
    s = torch.empty((count, n), device=dev)
    deg = torch.zeros((count, wsi), dtype=torch.int32, device=dev)
    out["mirror_degree_us"] = timed(lambda: nat.call("lds_bitmask_mirror_degree", P(bits1), n, W, count, P(deg), P(s),
                                                     st))
    # the factor all-gather's re-layout ([N, n, K] -> [n, N, K]) of U and V
    ug = torch.randn((N, n, K), generator=g, device=dev)
    out["factor_relayout_us"] = 2 * timed(lambda: ug.permute(1, 0, 2).contiguous())
    out["bytes_per_rank"] = {
        "dense_allreduce_ring_MB": 2 * (N - 1) / N * 4 * m / 1e6,
        "factor_allgather_received_MB": (N - 1) * (2 * n * K + n) * 4 / 1e6,
        "band_rows_sent_MB_max": max(v["sent_MB"] for v in bands.values()),
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
