"""Per-kernel floor inside a torch-captured HIP graph of ctypes launches:
K x lds_engine_advance (1 thread) and K x lds_sgd_clamp on 64 elements."""
import os, sys, time
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", ".."), os.path.join(os.path.dirname(__file__), "..", "..", "lds-gnn_amd")]
import torch
import ldsgnn
from ldsgnn import _native as nat

K = 200
sc = torch.zeros(32, dtype=torch.uint8, device="cuda")
a = torch.rand(64, device="cuda"); b = torch.rand(64, device="cuda")
big = torch.rand(1 << 20, device="cuda"); bigg = torch.rand(1 << 20, device="cuda")

def chain(kind):
    st = nat.stream_of(a.device)
    for _ in range(K):
        if kind == "advance":
            nat.call("lds_engine_advance", nat.ptr(sc), 1, 1, 1, 1, st)
        elif kind == "sgd64":
            nat.call("lds_sgd_clamp", nat.ptr(a), nat.ptr(b), 0.0, 64, st)
        elif kind == "sgd1M":
            nat.call("lds_sgd_clamp", nat.ptr(big), nat.ptr(bigg), 0.0, 1 << 20, st)
        elif kind == "torch_add":
            a.add_(b, alpha=0.0)

for kind in ["advance", "sgd64", "sgd1M", "torch_add"]:
    chain(kind); torch.cuda.synchronize()
    t0 = time.perf_counter(); chain(kind); torch.cuda.synchronize(); te = (time.perf_counter() - t0) / K * 1e6
    s = torch.cuda.Stream(); s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            chain(kind)
    torch.cuda.current_stream().wait_stream(s)
    g.replay(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5): g.replay()
    torch.cuda.synchronize(); tg = (time.perf_counter() - t0) / (5 * K) * 1e6
    print(f"{kind:10s} eager {te:6.2f} us/kernel   graph {tg:6.2f} us/kernel")
