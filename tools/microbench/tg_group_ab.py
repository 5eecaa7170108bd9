"""Config-5 θ-grad + SGD + next-window draw (lds_theta_grad_sgd_draw, the
128-tile form in XCD-grouped order, form 5) timed as a dependent chain, with a
checksum of θ, bits and degrees so that library builds with a different tile
order (kGroup in csrc/thetagrad.hip; load one with LDSGNN_LIB=path) can be
compared for identical results.  One JSON line.
Usage (GPU box): [LDSGNN_LIB=...] python tools/microbench/tg_group_ab.py [form]"""
import hashlib
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
from tg_draw_ab import chain_us  # noqa: E402


def main():
    form = sys.argv[1] if len(sys.argv) > 1 else "bf16x3-t128-grouped"
    n, k, graphs = 20000, 264, 6
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(n + k)
    u = torch.randn((n, k), generator=g, device=dev) * 0.01
    v = torch.randn((n, k), generator=g, device=dev) * 0.01
    r = torch.randn(n, generator=g, device=dev) * 0.01
    theta0 = torch.rand(n * (n + 1) // 2, generator=g, device=dev)
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
    prev = ops.theta_grad_form(form)

    def call(keep_grad=True):
        nat.call("lds_theta_grad_sgd_draw", nat.ptr(u), nat.ptr(v), k, k, nat.ptr(r), 1, 1, nat.ptr(theta), n,
                 nat.ptr(grad) if keep_grad else 0, nat.ptr(scal), seed, tag, nat.ptr(base), 0, graphs,
                 nat.ptr(bits), words, nat.ptr(deg), ops.form_code(), nat.stream_of(dev))
    call()
    torch.cuda.synchronize()
    h = hashlib.sha256()
    for t in (theta, grad, bits, deg):
        h.update(t.cpu().numpy().tobytes())

    def fn():
        call()
        deg.zero_()
    t = chain_us(fn, dev, copies=5, reps=4) - chain_us(lambda: deg.zero_(), dev, copies=5, reps=4)
    t_ng = chain_us(lambda: (call(False), deg.zero_()), dev, copies=5, reps=4) - \
        chain_us(lambda: deg.zero_(), dev, copies=5, reps=4)
    ops.theta_grad_form(prev)
    print(json.dumps({"lib": os.environ.get("LDSGNN_LIB", "default"), "form": form, "n": n, "k": k,
                      "graphs": graphs, "chain_us": t, "chain_us_no_grad_store": t_ng,
                      "checksum": h.hexdigest()[:16]}), flush=True)


if __name__ == "__main__":
    main()
