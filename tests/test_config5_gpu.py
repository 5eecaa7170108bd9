"""BASELINE config 5 at its full size (N = 20 000, θ_ij ~ U(0, 1) i.i.d., ≈2·10⁸
sampled entries per graph), through size-independent properties — the dense
oracle cannot run here (N² = 4·10⁸ fp32 per matrix, N³ normalisation):

  * θ-grad assembly (128-tile, XCD-grouped, 32-bit packed-index epilogue —
    the path config 5 takes) vs an fp64 restatement on sampled rows, and the
    64-bit index path (form 7, taken past n = 46 340) on the same inputs;
  * the bitmask aggregation (int8 MFMA) vs the CSR row-block SpMM and
    an fp64 restatement on sampled rows of the same sampled graph;
  * the batched window sampler vs single draws (bit-exact);
  * a long-row engine window (bitmask aggregation pre-pass, no CSR) vs the
    in-kernel CSR aggregation engine from the same state.

Reference ops: src/utils/graph.py:136-153 (normalisation), src/models/
layers.py:44 (Â·Z), src/models/sampling.py:47-79 (the draw)."""
import numpy as np
import pytest
import torch

from ldsgnn import _native as nat
from ldsgnn import ops
from ldsgnn.rng import TAG_GRAPH, Generator, tag_for

pytestmark = pytest.mark.gpu
N = 20000
TOL = 1e-5


def _rows(n, k, seed):
    return torch.randperm(n, generator=torch.Generator().manual_seed(seed))[:k].tolist() + [0, n - 1]


@pytest.mark.parametrize("form", ["bf16x3", "bf16x3-t128-grouped-i64"])
def test_theta_grad_n20000_vs_fp64_rows(device, form):
    n, k, S = N, 264, 1
    g = torch.Generator(device=device).manual_seed(n + k)
    u = torch.randn((n, k), generator=g, device=device)
    v = torch.randn((n, k), generator=g, device=device) * 0.1
    r = torch.randn((S, n), generator=g, device=device)
    m = n * (n + 1) // 2
    theta = torch.rand(m, generator=g, device=device)
    grad = torch.empty(m, device=device)
    scal = torch.zeros(32, dtype=torch.uint8, device=device)
    prev = ops.theta_grad_form(form)
    try:
        nat.call("lds_theta_grad_ex", nat.ptr(u), nat.ptr(v), k, k, nat.ptr(r), 1, n, S, nat.ptr(theta), n,
                 nat.ptr(grad), 0, nat.ptr(scal), 1.0, ops.form_code(), nat.stream_of(device))
        torch.cuda.synchronize()
    finally:
        ops.theta_grad_form(prev)
    ud, vd, rd = u.double(), v.double(), r.double().sum(0)
    for i in _rows(n, 10, 5):
        base = i * (2 * n - i + 1) // 2
        ref = ud[i] @ vd[i:].T + vd[i] @ ud[i:].T + rd[i] + rd[i:]
        ref[0] = 0.0  # diagonal
        got = grad[base:base + n - i].double()
        if i == n - 1:  # the last row is its diagonal alone: dθ_ii = 0
            assert float(got.abs().max()) == 0.0
            continue
        assert float((got - ref).abs().max() / ref.abs().max()) < TOL, (form, i)


@pytest.fixture(scope="module")
def dense_graph():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(20000)
    theta = torch.rand(N * (N + 1) // 2, generator=g, device=dev)
    graph = ops.sample_graph_from_triu(theta, N, generator=Generator(77), track_grad=False)
    del theta
    return graph


def test_bitmask_aggregation_n20000_vs_csr_and_fp64_rows(device, dense_graph):
    graph = dense_graph
    assert graph.nnz() > 1.9e8 and graph.long_rows()
    z = torch.randn(N, 16, generator=torch.Generator().manual_seed(3)).to(device)
    y_bit = graph.spmm_bitmask(z)
    y_csr = graph.spmm(z)  # long rows: the CSR spill-pass kernel (lds_spmm_norm_dense)
    torch.cuda.synchronize()
    rp = graph.row_ptr.cpu()
    zd = z.double().cpu()
    s = graph.s.double().cpu()
    for i in _rows(N, 6, 9):
        cols = graph.col[int(rp[i]):int(rp[i + 1])].long().cpu()
        ref = s[i] * (s[cols, None] * zd[cols]).sum(0)
        scale = (s[i] * (s[cols, None] * zd[cols]).abs().sum(0)).clamp(min=1e-30)
        assert float(((y_bit[i].double().cpu() - ref).abs() / scale).max()) < TOL, i
        assert float(((y_csr[i].double().cpu() - ref).abs() / scale).max()) < TOL, i
    colscale = (y_csr.abs().max(0).values.double() + 1e-30)
    assert float(((y_bit.double() - y_csr.double()).abs().max(0).values / colscale).max()) < TOL


def test_degrees_and_scale_n20000(device, dense_graph):
    """deg = row popcount of the bitmask (self-loop set), s = deg^-1/2 correctly
    rounded, row_ptr = exclusive scan of deg."""
    graph = dense_graph
    deg = graph.deg.long()
    assert torch.equal(graph.row_ptr[1:].long() - graph.row_ptr[:-1].long(), deg)
    want = np.float32(1.0) / np.sqrt(deg.cpu().numpy().astype(np.float32))  # IEEE fp32, correctly rounded
    assert np.array_equal(graph.s.cpu().numpy().view(np.uint32), want.view(np.uint32))
    pc = torch.zeros(N, dtype=torch.int64, device=device)
    for w in range((N + 63) // 64):  # the row's words (the stride pads to an even count)
        x = graph.bits[:, w]
        for k in range(64):
            pc += (x >> k) & 1
    assert torch.equal(pc, deg)


def test_batched_sampler_n20000_equals_single_draws(device):
    n, count = N, 2
    g = torch.Generator(device=device).manual_seed(n)
    theta = torch.rand(n * (n + 1) // 2, generator=g, device=device)
    words = nat.lib.lds_bitmask_words(n)
    st = nat.stream_of(device)
    base = torch.tensor([3, 0, 0, 0], dtype=torch.int32, device=device)
    bits = torch.empty((count, 1, n, words), dtype=torch.int64, device=device)
    deg = torch.empty((count, 1, nat.lib.lds_sample_ws_ints(n)), dtype=torch.int32, device=device)
    s = torch.empty((count, 1, n), dtype=torch.float32, device=device)
    seed, tag = 99, tag_for(TAG_GRAPH, 0)
    nat.call("lds_sample_graphs_multi", nat.ptr(theta), n, seed, tag, 1, nat.ptr(base), 1, count, 1,
             nat.ptr(bits), words, nat.ptr(deg), 0, 0, 0, nat.ptr(s), 0, 0, 0, 0, st)
    one = torch.empty((n, words), dtype=torch.int64, device=device)
    nb = (n + 63) // 64
    for gi in range(count):
        nat.call("lds_sample_bitmask", nat.ptr(theta), n, seed, tag, 3 + 1 + gi, 0, nat.ptr(one), words, st)
        assert torch.equal(bits[gi, 0, :, :nb], one[:, :nb]), gi


def test_long_row_window_n20000_matches_in_kernel_aggregation(device):
    """One τ = 2 window of the config-5 engine (long rows: bitmask aggregation
    pre-pass, no CSR) against the short-row engine (in-kernel CSR
    aggregation, n² column capacity) from the same state: losses, weights
    and θ on sampled entries."""
    from ldsgnn.data.workloads import load_workload
    from ldsgnn.engine import LdsEngine
    from ldsgnn.rng import Generator as Gen
    data = load_workload("synthetic20k", seed=1, device=device)
    n = data.num_nodes
    from ldsgnn.utils.graph import get_triu_values
    theta0 = get_triu_values(data.dense_adj).contiguous()
    del data.dense_adj
    torch.cuda.empty_cache()
    opt = data.val_mask.clone()
    opt[torch.nonzero(opt).squeeze(1)[::2]] = False
    res = []
    for long_rows in (True, False):
        torch.manual_seed(4)
        from oracle import lds_oracle as O
        params = O.init_params(data.num_features, 16, data.num_classes)
        params = {k: v.to(device) for k, v in params.items()}
        eng = LdsEngine(data.x, data.y, data.train_mask, opt, theta0.clone(), data.num_classes, dropout=0.5,
                        outer_lr=0.1, lr_decay=0.99, tau=2, generator=Gen(11, 0), params=params,
                        long_rows=long_rows)
        assert eng.long_rows == long_rows
        eng.run_window(2)
        torch.cuda.synchronize()
        res.append(dict(loss=[eng.inner_metrics(t)[0] for t in range(2)] + [eng.outer_metrics()[0]],
                        params=torch.cat([p.reshape(-1) for p in eng.get_params().values()]).cpu(),
                        theta=eng.theta[::997].cpu(), grad=eng.grad[::997].cpu()))
        del eng
        torch.cuda.empty_cache()
    a, b = res
    assert np.allclose(a["loss"], b["loss"], rtol=TOL, atol=1e-6)
    assert torch.allclose(a["params"], b["params"], rtol=TOL, atol=1e-6)
    gs = float(b["grad"].abs().max())
    assert float((a["grad"] - b["grad"]).abs().max()) < 1e-4 * gs
    assert torch.allclose(a["theta"], b["theta"], rtol=TOL, atol=1e-6)


def test_spmm_dense_n20000_vs_bitmask_csr_and_fp64_rows(device, dense_graph):
    """The config-5 CSR-SpMM (lds_spmm_norm_dense: the CSR index stream into
    bit rows, int8 matrix-core product) on the full-size sampled graph:
    against fp64 rows, the bitmask aggregation and the column-blocked CSR
    kernel, repeatable bit for bit and equal to the round-3 tile kernel."""
    graph = dense_graph
    z = torch.randn(N, 16, generator=torch.Generator().manual_seed(3)).to(device)
    ws = torch.empty(int(nat.lib.lds_spmm_dense_ws_bytes(N)), dtype=torch.uint8, device=device)
    err = torch.zeros(1, dtype=torch.int32, device=device)
    outs = []
    for _ in range(2):
        y = torch.empty(N, 16, device=device)
        nat.call("lds_spmm_norm_dense", nat.ptr(graph.row_ptr), nat.ptr(graph.col), nat.ptr(graph.s), N, nat.ptr(z),
                 16, nat.ptr(y), 16, 0, nat.ptr(ws), 0, 1, nat.ptr(err), nat.stream_of(device))
        outs.append(y)
    y_tile = torch.empty(N, 16, device=device)  # the round-3 tile kernel (grid < 0): the same exact sums
    nat.call("lds_spmm_norm_dense", nat.ptr(graph.row_ptr), nat.ptr(graph.col), nat.ptr(graph.s), N, nat.ptr(z),
             16, nat.ptr(y_tile), 16, 0, nat.ptr(ws), -256, 1, 0, nat.stream_of(device))
    torch.cuda.synchronize()
    assert int(err.item()) == 0  # the sampler's canonical CSR: no column-order flag
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(outs[0], y_tile)
    y = outs[0]
    y_bit = graph.spmm_bitmask(z)
    y_csr = graph.spmm(z)
    rp = graph.row_ptr.cpu()
    zd = z.double().cpu()
    s = graph.s.double().cpu()
    for i in _rows(N, 6, 11):
        cols = graph.col[int(rp[i]):int(rp[i + 1])].long().cpu()
        ref = s[i] * (s[cols, None] * zd[cols]).sum(0)
        scale = (s[i] * (s[cols, None] * zd[cols]).abs().sum(0)).clamp(min=1e-30)
        assert float(((y[i].double().cpu() - ref).abs() / scale).max()) < TOL, i
    colscale = (y_csr.abs().max(0).values.double() + 1e-30)
    assert float(((y.double() - y_csr.double()).abs().max(0).values / colscale).max()) < TOL
    assert float(((y.double() - y_bit.double()).abs().max(0).values / colscale).max()) < TOL


@pytest.mark.parametrize("kernel", ["bitmask", "csr"])
def test_long_row_outer_only_n20000_at_north_star_tolerance(device, kernel):
    """Config 5 at full size, the long-row kernels' θ-gradient at the
    north-star 1e-5 × max|dθ| (the well-conditioned construction of the
    config-2 golden hypergrad_cora_wellcond): dropout-free, a hyper step whose
    window has no inner step (every aggregation of the outer graph's forward
    and backward on the long-row kernel: the bitmask aggregation or the CSR
    spill-pass SpMM), against the short-row engine (in-kernel CSR
    aggregation) from the same state, on every 997th entry of dθ; θ after it
    within 1e-5."""
    from ldsgnn.data.workloads import load_workload
    from ldsgnn.engine import LdsEngine
    from ldsgnn.rng import Generator as Gen
    from ldsgnn.utils.graph import get_triu_values
    from oracle import lds_oracle as O
    data = load_workload("synthetic20k", seed=1, device=device)
    theta0 = get_triu_values(data.dense_adj).contiguous()
    del data.dense_adj
    torch.cuda.empty_cache()
    opt = data.val_mask.clone()
    opt[torch.nonzero(opt).squeeze(1)[::2]] = False
    res = []
    for long_rows in (True, False):
        torch.manual_seed(4)
        params = {k: v.to(device) for k, v in O.init_params(data.num_features, 16, data.num_classes).items()}
        eng = LdsEngine(data.x, data.y, data.train_mask, opt, theta0.clone(), data.num_classes, dropout=0.0,
                        outer_lr=0.1, lr_decay=0.99, tau=2, generator=Gen(13, 0), params=params,
                        long_rows=long_rows, long_rows_kernel=kernel)
        assert eng.long_rows == long_rows
        eng.hyper_step()  # θ₀'s outer graph only (no inner step in the window)
        torch.cuda.synchronize()
        res.append(dict(loss=eng.outer_metrics()[0], grad=eng.grad[::997].cpu(), theta=eng.theta[::997].cpu()))
        del eng
        torch.cuda.empty_cache()
    a, b = res
    assert abs(a["loss"] - b["loss"]) <= TOL * abs(b["loss"])
    gs = float(b["grad"].abs().max())
    err = float((a["grad"] - b["grad"]).abs().max())
    print(f"config 5 [{kernel}] outer-only dθ error / max|dθ|: {err / gs:.2e}")
    assert err <= 1e-5 * gs, (kernel, err / gs)
    assert torch.allclose(a["theta"], b["theta"], rtol=TOL, atol=1e-6)
