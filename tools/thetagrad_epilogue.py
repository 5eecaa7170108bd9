"""Split a θ-grad assembly launch into its parts: the same call with k = 0
(R terms and the fused SGD epilogue only: θ read, θ and grad written) against
the full k, per form, at config 5's n = 20 000 and Cora's n = 2708."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "lds-gnn_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402

from ldsgnn import _native as nat  # noqa: E402
from ldsgnn import ops  # noqa: E402
from thetagrad_forms import time_it  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    for n, kfull, reps in [(20000, 264, 5), (2708, 264, 50)]:
        m = n * (n + 1) // 2
        u = torch.randn((n, kfull), device=dev)
        v = torch.randn((n, kfull), device=dev)
        r = torch.randn((1, n), device=dev)
        theta = torch.rand(m, device=dev)
        grad = torch.empty(m, device=dev)
        scal = torch.zeros(32, dtype=torch.uint8, device=dev)
        scal[16:24].view(torch.float64).fill_(1e-9)
        st = nat.stream_of(dev)
        res = {"n": n}
        for form in ("fp32", "bf16x3-t64k16", "bf16x3-t128-grouped"):
            ops.theta_grad_form(form)
            for k in (0, 8, kfull):
                for gp in (True, False):
                    gptr = nat.ptr(grad) if gp else 0
                    t = time_it(lambda: nat.call("lds_theta_grad_ex", nat.ptr(u), nat.ptr(v), kfull, k, nat.ptr(r), 1,
                                                 n, 1, nat.ptr(theta), n, gptr, 2, nat.ptr(scal), 1.0, ops.form_code(), st), reps)
                    res[f"{form}/k{k}/{'grad' if gp else 'nograd'}"] = round(t, 1)
        ops.theta_grad_form("bf16x3")
        res["epilogue_bytes_grad"] = 12 * m
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
