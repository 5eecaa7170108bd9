"""Kernel-level parity of the HIP hot path against the CPU oracle.

Bit-exact for integer / index / RNG work (Philox uniforms, sampled edge sets,
CSR, degrees, s = deg^-1/2, dropout masks); fp32 kernels within the tolerance
BASELINE.json's north_star states (1e-5), stated per test.
"""
import numpy as np
import pytest
import torch

import ldsgnn
from ldsgnn import _native as nat
from ldsgnn import ops
from ldsgnn.rng import Generator, TAG_GRAPH, tag_for
from oracle import philox

pytestmark = pytest.mark.gpu

RTOL = 1e-5


def expected_graph(theta_np: np.ndarray, n: int, u: np.ndarray):
    """Oracle: A_ij = u_ij < clamp(θ_ij) for i < j, symmetric, self-loops set."""
    iu = np.triu_indices(n)
    p = np.zeros((n, n), dtype=np.float32)
    p[iu] = np.clip(theta_np, 0.0, 1.0)
    a = (u < p)
    a = np.triu(a, 1)
    a = a | a.T
    np.fill_diagonal(a, True)
    deg = a.sum(1).astype(np.int32)
    row_ptr = np.zeros(n + 1, dtype=np.int64)
    row_ptr[1:] = np.cumsum(deg)
    col = np.nonzero(a)[1].astype(np.int32)
    s = np.float32(1.0) / np.sqrt(deg.astype(np.float32))
    return a, deg, row_ptr, col, s


def bits_to_dense(bits: torch.Tensor, n: int) -> np.ndarray:
    b = bits.cpu().numpy().view(np.uint64)
    out = np.zeros((n, n), dtype=bool)
    for w in range((n + 63) // 64):
        word = b[:, w]
        for k in range(64):
            j = 64 * w + k
            if j < n:
                out[:, j] = (word >> np.uint64(k)) & np.uint64(1)
    return out


def test_philox_uniform_bit_exact(device):
    for rows, cols, seed, tag, ctr in [(37, 101, 123, 5, 0), (4, 4, 2**40 + 7, 1 << 24, 9), (130, 3, 0, 0, 77)]:
        got = ops.philox_uniform(seed, tag, ctr, rows, cols, device).cpu().numpy()
        want = philox.uniform(seed, tag, ctr, rows, cols)
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("n", [1, 2, 3, 63, 64, 65, 130, 300])
def test_sampler_bit_exact_vs_oracle(device, n):
    g = torch.Generator().manual_seed(n)
    theta = torch.rand(n * (n + 1) // 2, generator=g)
    gen = Generator(seed=1234 + n, replica=3)
    graph = ops.sample_graph_from_triu(theta.to(device), n, generator=gen, track_grad=False)
    u = philox.uniform(1234 + n, tag_for(TAG_GRAPH, 3), 0, n, n)
    a, deg, row_ptr, col, s = expected_graph(theta.numpy(), n, u)
    assert np.array_equal(bits_to_dense(graph.bits, n), a)
    assert np.array_equal(graph.deg.cpu().numpy(), deg)
    assert np.array_equal(graph.row_ptr.cpu().numpy(), row_ptr)
    assert graph.nnz() == len(col)
    assert np.array_equal(graph.col[: len(col)].cpu().numpy(), col)
    assert np.array_equal(graph.s.cpu().numpy().view(np.uint32), s.view(np.uint32))
    assert gen.graph_counter == 1


def test_sampler_injected_uniforms_match_torch_bernoulli(device):
    """Injected-U mode reproduces the reference's own draw:
    Bernoulli(P).sample() under torch.manual_seed (src/models/sampling.py:68)."""
    n = 200
    g = torch.Generator().manual_seed(7)
    theta = torch.rand(n * (n + 1) // 2, generator=g)
    iu = torch.triu_indices(n, n)
    p = torch.zeros(n, n)
    p[iu[0], iu[1]] = theta
    p = (p.triu(1) + p.triu(1).t() + torch.diag(p.diag())).clamp(0, 1)
    torch.manual_seed(99)
    ref = torch.distributions.Bernoulli(probs=p).sample()
    ref = ref.triu(1) + ref.triu(1).t()
    ref.fill_diagonal_(1.0)
    torch.manual_seed(99)
    u = torch.rand(n, n)
    graph = ops.sample_graph_from_triu(theta.to(device), n, u_inject=u.to(device), track_grad=False)
    assert torch.equal(graph.to_dense().cpu(), ref)


def test_sampler_known_answers(device):
    """θ ∈ {0, 1} is deterministic (tst/models/test_sampling.py:149-160)."""
    n = 70
    ones = torch.ones(n * (n + 1) // 2, device=device)
    full = ops.sample_graph_from_triu(ones, n, generator=Generator(5), track_grad=False)
    assert torch.equal(full.to_dense().cpu(), torch.ones(n, n))
    assert full.num_edges() == n * (n - 1) // 2
    zeros = torch.zeros_like(ones)
    empty = ops.sample_graph_from_triu(zeros, n, generator=Generator(5), track_grad=False)
    assert torch.equal(empty.to_dense().cpu(), torch.eye(n))
    assert torch.equal(empty.s.cpu(), torch.ones(n))
    # out-of-range θ is clamped like triu_values_to_symmetric_matrix
    big = ops.sample_graph_from_triu(ones * 3.0, n, generator=Generator(5), track_grad=False)
    assert big.num_edges() == n * (n - 1) // 2


@pytest.mark.parametrize("f", [1, 7, 16, 33, 64])
def test_spmm_norm_vs_dense(device, f):
    n = 333
    g = torch.Generator().manual_seed(f)
    theta = torch.rand(n * (n + 1) // 2, generator=g) * 0.2
    graph = ops.sample_graph_from_triu(theta.to(device), n, generator=Generator(f), track_grad=False)
    z = torch.randn(n, f, generator=g)
    y = graph.spmm(z.to(device)).cpu().double()
    a_hat = graph.normalized_dense().cpu().double()
    ref = a_hat @ z.double()
    assert torch.allclose(y, ref, rtol=RTOL, atol=RTOL)
    # strided input / beta=1 accumulate
    zz = torch.randn(n, f + 5, generator=g).to(device)
    out = torch.ones(n, f + 3, device=device)
    graph.spmm(zz[:, :f], out=out[:, :f], beta=1)
    ref2 = a_hat @ zz[:, :f].cpu().double() + 1.0
    assert torch.allclose(out[:, :f].cpu().double(), ref2, rtol=RTOL, atol=RTOL)
    assert torch.equal(out[:, f:].cpu(), torch.ones(n, 3))


@pytest.mark.parametrize("n,k,nr", [(1, 4, 1), (64, 16, 2), (150, 20, 3), (257, 64, 4)])
def test_theta_grad_vs_dense(device, n, k, nr):
    g = torch.Generator().manual_seed(n + k)
    u = torch.randn(n, k, generator=g)
    v = torch.randn(n, k, generator=g)
    r = torch.randn(n, nr, generator=g)
    theta = torch.rand(n * (n + 1) // 2, generator=g)
    theta[::7] = 1.5  # outside [0,1]: clamp backward masks these
    out = ops.theta_grad(u.to(device), v.to(device), r.to(device), n, theta=theta.to(device)).cpu().double()
    ud, vd, rd = u.double(), v.double(), r.double().sum(1)
    m = ud @ vd.t() + vd @ ud.t() + rd[:, None] + rd[None, :]
    iu = torch.triu_indices(n, n)
    ref = m[iu[0], iu[1]]
    ref[iu[0] == iu[1]] = 0.0
    ref[(theta.double() < 0) | (theta.double() > 1)] = 0.0
    assert torch.allclose(out, ref, rtol=RTOL, atol=1e-4)
    # accumulate
    base = torch.randn(n * (n + 1) // 2, generator=g)
    acc = base.clone().to(device)
    ops.theta_grad(u.to(device), v.to(device), r.to(device), n, theta=theta.to(device), out=acc, accumulate=True)
    assert torch.allclose(acc.cpu().double(), base.double() + ref, rtol=RTOL, atol=1e-4)


def test_dropout_bit_exact(device):
    rows, cols = 37, 50
    x = torch.randn(rows, cols)
    key = (99, tag_for(2 << 24, 1), 4)
    y = ops.keyed_dropout(x.to(device), 0.5, key).cpu()
    u = philox.uniform(99, key[1], 4, rows, cols)
    ref = x * torch.from_numpy((u < 0.5).astype(np.float32)) * 2.0
    assert torch.equal(y, ref)


def test_sgd_clamp(device):
    g = torch.Generator().manual_seed(0)
    for count in [1, 5, 1000, 4097]:
        th = torch.rand(count, generator=g)
        gr = torch.randn(count, generator=g)
        t = th.to(device)
        ops.sgd_clamp_(t, gr.to(device), 0.3)
        ref = (th - 0.3 * gr).clamp(0, 1)
        assert torch.allclose(t.cpu(), ref, atol=1e-6)


def test_native_errors_are_raised(device):
    with pytest.raises(nat.NativeError):
        nat.call("lds_spmm_norm", 0, 0, 0, 10, 0, 4, 4, 0, 4, 0, 0)


def test_degree_scale_is_correctly_rounded(device):
    """s = fl32(1/fl32(sqrt(d))) bit-exact for every degree 1..20000."""
    n = 20000
    deg = torch.arange(1, n + 1, dtype=torch.int64)
    row_ptr = torch.zeros(n + 1, dtype=torch.int64)
    row_ptr[1:] = torch.cumsum(deg, 0)
    rp = row_ptr.to(torch.int32).to(device)
    s = torch.empty(n, device=device)
    d = torch.empty(n, dtype=torch.int32, device=device)
    nat.call("lds_csr_degree_scale", nat.ptr(rp), n, nat.ptr(d), nat.ptr(s), nat.stream_of(s.device))
    want = np.float32(1.0) / np.sqrt(deg.numpy().astype(np.float32))
    assert np.array_equal(d.cpu().numpy(), deg.numpy())
    assert np.array_equal(s.cpu().numpy().view(np.uint32), want.view(np.uint32))


def test_theta_grad_mfma_matches_valu_and_sgd_mode(device):
    """MFMA and VALU forms agree; the fused SGD mode equals grad-then-update."""
    n, k = 200, 40
    g = torch.Generator().manual_seed(1)
    u = torch.randn(n, k, generator=g).to(device)
    v = torch.randn(n, k, generator=g).to(device)
    r = torch.randn(n, 2, generator=g).to(device)
    theta = torch.rand(n * (n + 1) // 2, generator=g).to(device)
    a = ops.theta_grad(u, v, r, n, theta=theta)
    b = torch.empty_like(a)
    nat.call("lds_theta_grad_valu", nat.ptr(u), nat.ptr(v), k, k, nat.ptr(r), 2, 2, nat.ptr(theta), n, nat.ptr(b),
             0, nat.stream_of(u.device))
    assert torch.allclose(a, b, rtol=1e-5, atol=1e-5)
    sc = torch.zeros(32, dtype=torch.uint8, device=device)
    sc[16:24].view(torch.float64).fill_(0.3)
    th2 = theta.clone()
    gout = torch.empty_like(theta)
    nat.call("lds_theta_grad_sgd", nat.ptr(u), nat.ptr(v), k, k, nat.ptr(r), 2, 2, nat.ptr(th2), n, nat.ptr(gout),
             nat.ptr(sc), ops.form_code(), nat.stream_of(u.device))
    assert torch.equal(gout, a)
    assert torch.allclose(th2, (theta - 0.3 * a).clamp(0, 1), atol=1e-6)


@pytest.mark.parametrize("n,high", [(100, 1.0), (1500, 1.0), (2600, 0.5), (3000, 0.02)])
def test_spmm_blocked_vs_dense(device, n, high):
    """Column-blocked LDS SpMM (long rows, config 5's kernel) vs the dense fp64
    product: a graph smaller than one block, a complete graph (segments longer
    than one index chunk), dense random rows, and sparse rows (mostly empty
    segments).  Summation order differs from the CSR order: fp32 tolerance."""
    g = torch.Generator().manual_seed(n)
    theta = torch.rand(n * (n + 1) // 2, generator=g) * high
    graph = ops.sample_graph_from_triu(theta.to(device), n, generator=Generator(n), track_grad=False)
    z = torch.randn(n, 16, generator=g).to(device)
    y_blk = graph.spmm(z, blocked=True).cpu().double()
    y_row = graph.spmm(z, blocked=False).cpu().double()
    y_def = graph.spmm(z).cpu().double()  # long rows: the CSR spill-pass kernel (lds_spmm_norm_dense)
    ref = graph.normalized_dense().cpu().double() @ z.cpu().double()
    scale = ref.abs().max()
    assert float((y_blk - ref).abs().max() / scale) < RTOL
    assert float((y_row - ref).abs().max() / scale) < RTOL
    assert float((y_def - ref).abs().max() / scale) < RTOL
    for blocked in (True, None):
        out = torch.ones(n, 16, device=device)
        graph.spmm(z, out=out, beta=1, blocked=blocked)
        assert float((out.cpu().double() - ref - 1.0).abs().max() / scale) < RTOL, blocked


@pytest.mark.parametrize("n,high", [(1, 1.0), (65, 1.0), (700, 1.0), (1500, 1.0), (2600, 0.5), (3000, 0.02)])
def test_bitmask_agg_vs_dense(device, n, high):
    """Bitmask aggregation on the int8 matrix cores (lds_aggregate_bitmask) vs
    the dense fp64 product and the CSR kernel: ragged n (not a multiple of the
    64-row tile or the 512-column chunk), complete, dense and sparse graphs.
    Per-column tolerance 1e-5 of max_i Σ_k |Â_ik z_kf| (the quantisation is
    2^-31 of the column maximum; integer sums are exact)."""
    g = torch.Generator().manual_seed(n + 17)
    theta = torch.rand(n * (n + 1) // 2, generator=g) * high
    graph = ops.sample_graph_from_triu(theta.to(device), n, generator=Generator(n), track_grad=False)
    z = torch.randn(n, 16, generator=g)
    z[:, 3] *= 1e-30   # tiny column
    z[:, 7] *= 1e30    # huge column
    z[:, 11] = 0.0     # empty column
    z[: n // 2, 13] *= 1e6   # dynamic range inside a column
    zd = z.to(device)
    y = graph.spmm_bitmask(zd).cpu().double()
    a = graph.normalized_dense().cpu().double()
    ref = a @ z.double()
    scale = (a.abs() @ z.double().abs()).max(0).values.clamp(min=1e-300)
    assert float(((y - ref).abs().max(0).values / scale).max()) < RTOL
    assert torch.all(y[:, 11] == 0)
    y_csr = graph.spmm(zd, blocked=False).cpu().double()
    assert float(((y - y_csr).abs().max(0).values / scale).max()) < RTOL
    # beta = 1 and strided Z / Y
    zs = torch.zeros(n, 24, device=device)
    zs[:, :16] = zd
    out = torch.ones(n, 20, device=device)
    ws = torch.empty(int(nat.lib.lds_bitmask_agg_ws_bytes(n)), dtype=torch.uint8, device=device)
    nat.call("lds_aggregate_bitmask", nat.ptr(graph.bits), graph.bits.size(1), nat.ptr(graph.s), n, nat.ptr(zs), 24,
             nat.ptr(out), 20, 1, nat.ptr(ws), nat.stream_of(zd.device))
    o = out.cpu().double()
    assert float(((o[:, :16] - ref - 1.0).abs().max(0).values / scale.clamp(min=1.0)).max()) < RTOL
    assert torch.all(o[:, 16:] == 1.0)


@pytest.mark.parametrize("n", [65, 1500, 3000])
def test_bitmask_agg_repeatable_on_dirty_workspace(device, n):
    """A workspace full of garbage and back-to-back calls give bit-identical
    Y: one split (n = 65: y written by the main kernel) and several (the
    split partials summed in fixed order by the final launch)."""
    g = torch.Generator().manual_seed(n + 5)
    theta = torch.rand(n * (n + 1) // 2, generator=g)
    graph = ops.sample_graph_from_triu(theta.to(device), n, generator=Generator(n), track_grad=False)
    z = torch.randn(n, 16, generator=g).to(device)
    ws = torch.full((int(nat.lib.lds_bitmask_agg_ws_bytes(n)),), 0x7F, dtype=torch.uint8, device=device)
    outs = []
    for _ in range(3):
        y = torch.empty(n, 16, device=device)
        nat.call("lds_aggregate_bitmask", nat.ptr(graph.bits), graph.bits.size(1), nat.ptr(graph.s), n, nat.ptr(z),
                 16, nat.ptr(y), 16, 0, nat.ptr(ws), nat.stream_of(z.device))
        outs.append(y.cpu())
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    ref = graph.normalized_dense().cpu().double() @ z.cpu().double()
    assert float((outs[0].double() - ref).abs().max() / ref.abs().max()) < RTOL


@pytest.mark.parametrize("n", [65, 1500, 3000])
def test_bitmask_agg_partials_fold_bit_exact(device, n):
    """lds_aggregate_bitmask_partials leaves the split partial sums; a consumer
    forming s_i · Σ_p part_p[i] in split order (what the engine kernels do with
    LdsBatch.agg_splits) reproduces lds_aggregate_bitmask's y bit for bit."""
    g = torch.Generator().manual_seed(n + 7)
    theta = torch.rand(n * (n + 1) // 2, generator=g)
    graph = ops.sample_graph_from_triu(theta.to(device), n, generator=Generator(n), track_grad=False)
    z = torch.randn(n, 16, generator=g).to(device)
    st = nat.stream_of(z.device)
    ws = torch.empty(int(nat.lib.lds_bitmask_agg_ws_bytes(n)), dtype=torch.uint8, device=device)
    y = torch.empty(n, 16, device=device)
    nat.call("lds_aggregate_bitmask", nat.ptr(graph.bits), graph.bits.size(1), nat.ptr(graph.s), n, nat.ptr(z), 16,
             nat.ptr(y), 16, 0, nat.ptr(ws), st)
    ws2 = torch.full_like(ws, 0x55)
    nat.call("lds_aggregate_bitmask_partials", nat.ptr(graph.bits), graph.bits.size(1), nat.ptr(graph.s), n,
             nat.ptr(z), 16, nat.ptr(ws2), st)
    ks = int(nat.lib.lds_bitmask_agg_splits(n))
    off = int(nat.lib.lds_bitmask_agg_part_offset(n))
    part = ws2[off:off + ks * n * 16 * 4].view(torch.float32).view(ks, n, 16)
    acc = torch.zeros(n, 16, device=device)
    for p in range(ks):  # in split order, as the consumers add them
        acc = acc + part[p]
    got = graph.s.view(n, 1) * acc
    torch.cuda.synchronize()
    assert torch.equal(got, y)


def test_pretrain_step_vs_oracle(device):
    """Fused pre-training epoch (weighted BCE + clamp/symmetrisation backward +
    Adam on packed θ, one launch) against the reference's dense restatement
    (oracle.pretrain_epoch_dense with torch.optim.Adam) over 6 epochs."""
    from oracle import lds_oracle as O
    from ldsgnn.trainers.pretrainer import edges_to_bits
    n = 150
    g = torch.Generator().manual_seed(21)
    theta0 = torch.rand(n * (n + 1) // 2, generator=g) * 1.2 - 0.1  # some entries outside [0, 1]
    a = (torch.rand(n, n, generator=g) < 0.05).float().triu(1)
    t = a + a.t()
    th_o = torch.nn.Parameter(theta0.clone())
    opt = torch.optim.Adam([th_o], lr=0.01)
    th_p = theta0.clone().to(device)
    m, v = torch.zeros_like(th_p), torch.zeros_like(th_p)
    bits = edges_to_bits(t.nonzero().t(), n, device)
    pos_weight = float(np.float32((n * n - t.sum().item()) / t.sum().item()))
    rows = torch.zeros(n, device=device)
    for step in range(1, 7):
        lo = O.pretrain_epoch_dense(th_o, t, opt)
        nat.call("lds_pretrain_step", nat.ptr(th_p), n, nat.ptr(bits), bits.size(1), pos_weight, nat.ptr(m),
                 nat.ptr(v), step, 0.01, 0.9, 0.999, 1e-8, nat.ptr(rows), nat.stream_of(th_p.device))
        lp = float(rows.double().sum().item()) / (n * n)
        assert abs(lp - lo) <= 1e-5 * abs(lo), (step, lp, lo)
        assert float((th_p.cpu() - th_o.detach()).abs().max()) < 1e-5, step


@pytest.mark.parametrize("n,k,mode", [(300, 520, 0), (129, 1030, 1), (257, 600, 2), (64, 512, 0)])
def test_theta_grad_ex_wide_k(device, n, k, mode):
    """lds_theta_grad_ex at wide k (the 128×128-tile kernel, replica samples):
    R stacked as S rows of n (ldr_col = n), gscale = 1/S, modes grad =, +=,
    and the fused SGD + clamp, vs the dense fp64 formula."""
    S = 3
    g = torch.Generator().manual_seed(n + k)
    u = torch.randn(n, k, generator=g)
    v = torch.randn(n, k, generator=g)
    r = torch.randn(S, n, generator=g)
    theta = torch.rand(n * (n + 1) // 2, generator=g)
    theta[::5] = 1.25
    gs = float(np.float32(1.0) / np.float32(S))
    ud, vd, rd = u.double(), v.double(), r.double().sum(0)
    m = gs * (ud @ vd.t() + vd @ ud.t() + rd[:, None] + rd[None, :])
    iu = torch.triu_indices(n, n)
    ref = m[iu[0], iu[1]]
    ref[iu[0] == iu[1]] = 0.0
    ref[(theta.double() < 0) | (theta.double() > 1)] = 0.0
    base = torch.randn(n * (n + 1) // 2, generator=g)
    grad = base.clone().to(device)
    th = theta.clone().to(device)
    lr = 0.05
    scal = torch.zeros(32, dtype=torch.uint8, device=device)
    scal[16:24].view(torch.float64).fill_(lr)
    ud_, vd_, rd_ = u.to(device), v.to(device), r.to(device)  # keep the device copies alive across the call
    nat.call("lds_theta_grad_ex", nat.ptr(ud_), nat.ptr(vd_), k, k, nat.ptr(rd_), 1, n, S, nat.ptr(th), n,
             nat.ptr(grad), mode, nat.ptr(scal), gs, ops.form_code(), nat.stream_of(th.device))
    torch.cuda.synchronize()
    tol = 1e-5 * float(ref.abs().max())
    if mode == 0:
        assert float((grad.cpu().double() - ref).abs().max()) < tol
    elif mode == 1:
        assert float((grad.cpu().double() - base.double() - ref).abs().max()) < tol
    else:
        assert float((grad.cpu().double() - ref).abs().max()) < tol
        want = (theta.double() - lr * ref).clamp(0, 1)
        assert float((th.cpu().double() - want).abs().max()) < 1e-5


@pytest.mark.parametrize("n,count,samples", [(300, 3, 2), (6000, 3, 1), (6000, 2, 2)])
def test_batched_sampler_equals_single_draws(device, n, count, samples):
    """lds_sample_graphs_multi (graph g draws counter base + g, sample b tag +
    b·tag_step) is bit-identical to single lds_sample_bitmask draws, in both
    launch forms: one block per (tile, graph) and, past the MALL (θ > 64 MB at
    n = 6000), one block per tile looping over every (graph, sample) on one θ
    load.  col = NULL (bitmask + degrees only) is accepted."""
    g = torch.Generator().manual_seed(n)
    theta = (torch.rand(n * (n + 1) // 2, generator=g) * 0.6).to(device)
    words = nat.lib.lds_bitmask_words(n)
    st = nat.stream_of(theta.device)
    base = torch.tensor([7, 0, 0, 0], dtype=torch.int32, device=device)
    bits = torch.empty((count, samples, n, words), dtype=torch.int64, device=device)
    wsi = nat.lib.lds_sample_ws_ints(n)
    deg = torch.empty((count, samples, wsi), dtype=torch.int32, device=device)
    s = torch.empty((count, samples, n), dtype=torch.float32, device=device)
    seed, tag = 1234, tag_for(TAG_GRAPH, 5)
    nat.call("lds_sample_graphs_multi", nat.ptr(theta), n, seed, tag, 1, nat.ptr(base), 2, count, samples,
             nat.ptr(bits), words, nat.ptr(deg), 0, 0, 0, nat.ptr(s), 0, 0, 0, 0, st)
    one = torch.empty((n, words), dtype=torch.int64, device=device)
    nb = (n + 63) // 64
    for gi in range(count):
        for b in range(samples):
            nat.call("lds_sample_bitmask", nat.ptr(theta), n, seed, tag + b, 7 + 2 + gi, 0, nat.ptr(one), words, st)
            assert torch.equal(bits[gi, b, :, :nb], one[:, :nb]), (gi, b)
            pc = torch.zeros(n, dtype=torch.int64, device=device)
            for w in range(nb):
                x = one[:, w]
                for k in range(64):
                    pc += (x >> k) & 1
            assert torch.equal(deg[gi, b, :n].long(), pc), (gi, b)

@pytest.mark.parametrize("n,count,samples", [(300, 2, 3), (2708, 1, 8), (2708, 2, 5), (2708, 6, 1), (300, 6, 1)])
def test_sgd_sample_split_equals_one_block_per_tile(device, n, count, samples):
    """lds_sgd_sample_graphs with its (graph, sample) items split over grid.z
    (tile counters given; at Cora n, 6 graphs × 8 samples: five blocks per
    tile of ten items; one sample: one block, the counters unused) against
    one block per tile (tile_ctr NULL):
    bit-identical θ, bits and degree counts over two chained calls, θ equal to
    lds_engine_sgd_clamp's, and the counters left zero."""
    g = torch.Generator().manual_seed(n + samples)
    m = n * (n + 1) // 2
    theta0 = torch.rand(m, generator=g).to(device)
    grads = [(torch.randn(m, generator=g) * 0.3).to(device) for _ in range(2)]
    words = nat.lib.lds_bitmask_words(n)
    wsi = nat.lib.lds_sample_ws_ints(n)
    st = nat.stream_of(theta0.device)
    scalars = torch.zeros(nat.lib.lds_engine_scalars_size(), dtype=torch.uint8, device=device)
    scalars[:4].view(torch.int32).fill_(9)  # graph counter
    scalars[16:24].view(torch.float64).fill_(0.37)  # lr
    G = count * samples
    tiles = torch.zeros(nat.lib.lds_sgd_tile_ints(n), dtype=torch.int32, device=device)
    outs = []
    for split in (False, True):
        theta = theta0.clone()
        got = []
        for k, gr in enumerate(grads):
            bits = torch.zeros((G, n, words), dtype=torch.int64, device=device)
            deg = torch.zeros((G, wsi), dtype=torch.int32, device=device)
            nat.call("lds_sgd_sample_graphs", nat.ptr(theta), nat.ptr(gr), nat.ptr(scalars), n, 4321,
                     tag_for(TAG_GRAPH, 3), 1, 2 + 5 * k, count, samples, nat.ptr(bits), words, nat.ptr(deg),
                     nat.ptr(tiles) if split else 0, st)
            got.append((theta.clone(), bits, deg))
        torch.cuda.synchronize()
        assert int(tiles.abs().sum()) == 0
        outs.append(got)
    for (ta, ba, da), (tb, bb, db) in zip(*outs):
        assert torch.equal(ta, tb)
        assert torch.equal(ba, bb)
        assert torch.equal(da, db)
    want = theta0.clone()
    for gr in grads:
        nat.call("lds_engine_sgd_clamp", nat.ptr(want), nat.ptr(gr), m, nat.ptr(scalars), st)
    torch.cuda.synchronize()
    assert torch.equal(outs[1][-1][0], want)


def test_sgd_sample_split_stale_tile_counter_sets_device_error(device):
    """Round-5 ADVICE: the split SGD + draw pass assumes its per-tile
    counters are zero on entry.  With counters left at a value past the
    tile's block count (a stale or shared workspace), a block counts past the
    tile's blocks and sets LDS_DEVERR_SGD_TILE_COUNTER in the engine's error
    word (EngineScalars.error, byte 32 of `scalars`) instead of passing
    silently; with clean counters the word stays zero."""
    n, count, samples = 600, 6, 8
    g = torch.Generator().manual_seed(5)
    m = n * (n + 1) // 2
    words = nat.lib.lds_bitmask_words(n)
    wsi = nat.lib.lds_sample_ws_ints(n)
    st = nat.stream_of(torch.device(device))
    for stale in (0, 1000):
        theta = torch.rand(m, generator=g).to(device)
        gr = (torch.randn(m, generator=g) * 0.3).to(device)
        scalars = torch.zeros(nat.lib.lds_engine_scalars_size(), dtype=torch.uint8, device=device)
        scalars[16:24].view(torch.float64).fill_(0.1)
        tiles = torch.full((nat.lib.lds_sgd_tile_ints(n),), stale, dtype=torch.int32, device=device)
        bits = torch.zeros((count * samples, n, words), dtype=torch.int64, device=device)
        deg = torch.zeros((count * samples, wsi), dtype=torch.int32, device=device)
        nat.call("lds_sgd_sample_graphs", nat.ptr(theta), nat.ptr(gr), nat.ptr(scalars), n, 99,
                 tag_for(TAG_GRAPH, 0), 1, 0, count, samples, nat.ptr(bits), words, nat.ptr(deg), nat.ptr(tiles), st)
        torch.cuda.synchronize()
        word = int(scalars[32:36].view(torch.int32).item())
        assert word == (nat.DEVERR_SGD_TILE_COUNTER if stale else 0), (stale, word)


@pytest.mark.parametrize("n", [64, 130, 700, 1100])
def test_bitmask_mirror_degree_completes_symmetric_graphs(device, n):
    """lds_bitmask_mirror_degree (the band-sharded exchange's owner step):
    from a symmetric bitmask with its strictly-lower words cleared it rebuilds
    every lower word (8 × 8 super-blocks of 64 × 64 bit transposes, partial
    super-blocks at the edge) and writes the degrees and s = deg^-1/2 the
    sampler's popcount pass gives."""
    g = torch.Generator().manual_seed(n)
    graphs = 3
    words = nat.lib.lds_bitmask_words(n)
    wsi = nat.lib.lds_sample_ws_ints(n)
    a = torch.rand((graphs, n, n), generator=g) < 0.3
    a = a.triu(1)
    a = a | a.transpose(1, 2) | torch.eye(n, dtype=torch.bool)[None]
    pad = torch.zeros((graphs, n, 64 * words), dtype=torch.bool)
    pad[:, :, :n] = a
    wts = (1 << torch.arange(64, dtype=torch.int64))
    full = (pad.view(graphs, n, words, 64).long() * wts).sum(-1)  # [graphs, n, words] (two's complement wraps)
    upper = full.clone()
    for r in range(n):
        upper[:, r, :r // 64] = 0  # strictly-lower words
    bits = upper.to(device)
    deg = torch.zeros((graphs, wsi), dtype=torch.int32, device=device)
    s = torch.zeros((graphs, n), device=device)
    nat.call("lds_bitmask_mirror_degree", nat.ptr(bits), n, words, graphs, nat.ptr(deg), nat.ptr(s),
             nat.stream_of(torch.device(device)))
    torch.cuda.synchronize()
    assert torch.equal(bits.cpu(), full)
    want_deg = a.sum(-1).to(torch.int32)
    assert torch.equal(deg[:, :n].cpu(), want_deg)
    ref_full = full.to(device)  # the sampler's own degree pass on the complete bits: the same s bit for bit
    for gi in range(graphs):
        d1 = torch.zeros(n, dtype=torch.int32, device=device)
        s1 = torch.zeros(n, device=device)
        nat.call("lds_bitmask_degree", nat.ptr(ref_full[gi]), n, words, nat.ptr(d1), nat.ptr(s1),
                 nat.stream_of(torch.device(device)))
        torch.cuda.synchronize()
        assert torch.equal(s[gi], s1) and torch.equal(deg[gi, :n], d1)


def test_fill_guard_pads_inflated_degrees(device):
    """lds_sample_graphs_multi promised a zero degree workspace (ws_zeroed =
    1) that is not: every row's count exceeds its drawn bits.  The fill
    writes the drawn columns, pads each row's remaining slots with the row
    index (col was garbage before), leaves no CSR position outside [0, n) and
    sets LDS_DEVERR_FILL_DEGREE in the error word; a consistent call leaves
    the word alone.  Counts short of the bits (one less per row) are flagged
    and every row writes only its own slots.  Both fill forms: 16-lane rows
    and whole-wave dense rows."""
    for n, dense in ((300, 0.3), (1500, 0.9)):
        g = torch.Generator().manual_seed(n)
        theta = (torch.rand(n * (n + 1) // 2, generator=g) * dense).to(device)
        words = nat.lib.lds_bitmask_words(n)
        wsi = nat.lib.lds_sample_ws_ints(n)
        st = nat.stream_of(theta.device)
        base = torch.zeros(4, dtype=torch.int32, device=device)
        bits = torch.empty((n, words), dtype=torch.int64, device=device)
        rp = torch.empty(n + 1, dtype=torch.int32, device=device)
        s = torch.empty(n, dtype=torch.float32, device=device)
        ell = torch.empty(n * 128, dtype=torch.int32, device=device)
        err = torch.zeros(1, dtype=torch.int32, device=device)
        cap = n * n
        outs = []
        for extra in (0, 5, -1):
            ws = torch.full((wsi,), extra, dtype=torch.int32, device=device)
            col = torch.full((cap,), 0x7FFFFFFF, dtype=torch.int32, device=device)
            nat.call("lds_sample_graphs_multi", nat.ptr(theta), n, 11, tag_for(TAG_GRAPH, 0), 1, nat.ptr(base), 0,
                     1, 1, nat.ptr(bits), words, nat.ptr(ws), nat.ptr(rp), nat.ptr(col), cap, nat.ptr(s),
                     nat.ptr(ell), 0, 1, nat.ptr(err), st)
            torch.cuda.synchronize()
            assert int(err.item()) == (1 if extra else 0), (n, extra)
            err.zero_()
            outs.append((rp.clone().long().cpu(), col.cpu(), ws[:n].long().cpu()))
        (rp0, col0, d0), (rp1, col1, d1), (rp2, col2, d2) = outs
        assert torch.equal(d1, d0 + 5)
        nnz = int(rp1[n])
        assert nnz == int(d0.sum()) + 5 * n
        assert int(col1[:nnz].min()) >= 0 and int(col1[:nnz].max()) < n
        for r in range(0, n, max(1, n // 37)):
            got = col1[int(rp1[r]):int(rp1[r + 1])]
            k = int(d0[r])
            assert torch.equal(got[:k], col0[int(rp0[r]):int(rp0[r + 1])]), r
            assert bool((got[k:] == r).all()), r
        # counts one short of the bits (flagged above): every row keeps to its own
        # slots — its first deg - 1 columns, ascending — never the next row's
        assert torch.equal(d2, d0 - 1)
        for r in range(n):
            got = col2[int(rp2[r]):int(rp2[r + 1])]
            assert torch.equal(got, col0[int(rp0[r]):int(rp0[r + 1]) - 1]), r



@pytest.mark.parametrize("n,count,samples,dense", [(300, 3, 2, 0.3), (1000, 2, 1, 0.05), (2100, 2, 1, 0.9)])
def test_fused_sampler_csr_equals_staged_path(device, n, count, samples, dense):
    """The two-launch CSR sampler (degrees counted by the tile kernel, the scan
    folded into the fill) against the staged path (draw -> popcount degrees /
    s -> scan -> fill + ELL head): bit-identical row_ptr, col, s and ELL, with
    a dirty workspace cleared by the call (ws_zeroed = 0) and with a zeroed one
    (ws_zeroed = 1).  dense = 0.9 takes the word-at-a-time fill of rows past
    1024 entries."""
    g = torch.Generator().manual_seed(n + count)
    theta = (torch.rand(n * (n + 1) // 2, generator=g) * dense).to(device)
    words = nat.lib.lds_bitmask_words(n)
    wsi = nat.lib.lds_sample_ws_ints(n)
    st = nat.stream_of(theta.device)
    base = torch.tensor([5, 0, 0, 0], dtype=torch.int32, device=device)
    G = count * samples
    cap = n * n
    seed, tag = 77, tag_for(TAG_GRAPH, 2)
    outs = []
    for zeroed in (0, 1):
        bits = torch.empty((G, n, words), dtype=torch.int64, device=device)
        ws = torch.full((G, wsi), 0 if zeroed else 7, dtype=torch.int32, device=device)
        rp = torch.empty((G, n + 1), dtype=torch.int32, device=device)
        col = torch.full((G, cap), -1, dtype=torch.int32, device=device)
        s = torch.empty((G, n), dtype=torch.float32, device=device)
        ell = torch.empty((G, n * 128), dtype=torch.int32, device=device)
        nat.call("lds_sample_graphs_multi", nat.ptr(theta), n, seed, tag, 1, nat.ptr(base), 1, count, samples,
                 nat.ptr(bits), words, nat.ptr(ws), nat.ptr(rp), nat.ptr(col), cap, nat.ptr(s), nat.ptr(ell), 0, zeroed, 0, st)
        outs.append((rp.clone(), col.clone(), s.clone(), ell.clone(), ws[:, :n].clone()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    rp, col, s, ell, deg = outs[0]
    for gi in range(count):
        for b in range(samples):
            k = gi * samples + b
            one = torch.empty((n, words), dtype=torch.int64, device=device)
            nat.call("lds_sample_bitmask", nat.ptr(theta), n, seed, tag + b, 5 + 1 + gi, 0, nat.ptr(one), words, st)
            d1 = torch.empty(n, dtype=torch.int32, device=device)
            s1 = torch.empty(n, dtype=torch.float32, device=device)
            rp1 = torch.empty(n + 1, dtype=torch.int32, device=device)
            col1 = torch.full((cap,), -1, dtype=torch.int32, device=device)
            ell1 = torch.empty(n * 128, dtype=torch.int32, device=device)
            nat.call("lds_bitmask_degree", nat.ptr(one), n, words, nat.ptr(d1), nat.ptr(s1), st)
            nat.call("lds_exclusive_scan", nat.ptr(d1), n, nat.ptr(rp1), st)
            nat.call("lds_bitmask_fill_csr_ell", nat.ptr(one), n, words, nat.ptr(rp1), nat.ptr(col1), cap, 0,
                     nat.ptr(s1), nat.ptr(ell1), st)
            assert torch.equal(deg[k], d1), (gi, b)
            assert torch.equal(rp[k], rp1), (gi, b)
            assert torch.equal(s[k], s1), (gi, b)
            nnz = int(rp1[n])
            assert torch.equal(col[k, :nnz], col1[:nnz]), (gi, b)
            assert torch.equal(ell[k], ell1), (gi, b)


@pytest.mark.parametrize("form", ["bf16x3", "bf16x3-t64k16", "bf16x3-t64k16-grouped", "bf16x3-t64k32",
                                  "bf16x3-t128", "bf16x3-t128-grouped", "bf16x3-t128-pipe", "bf16x3-t128-w8",
                                  "fp32"])
@pytest.mark.parametrize("n,k,ld,mode", [(1, 4, 4, 0), (65, 17, 17, 0), (130, 33, 35, 1), (200, 0, 4, 0),
                                         (257, 48, 48, 2), (300, 264, 264, 3), (129, 1030, 1032, 0),
                                         (1100, 40, 40, 3)])
def test_theta_grad_forms_vs_dense(device, form, n, k, ld, mode):
    """Every arithmetic form of the θ-grad assembly (fp32 MFMA; split-bf16 with
    32- and 16-wide k chunks) against the dense fp64 formula, across modes,
    ragged k (partial chunks and k-steps), an unaligned row stride (scalar
    staging), k = 0 (R only) and n = 1.  Tolerance 1e-5 × max |g| (north_star's
    fp32 tolerance; split-bf16 keeps products to ~2⁻²² relative)."""
    g = torch.Generator().manual_seed(7 * n + k)
    ub = torch.randn(n, ld, generator=g)
    vb = torch.randn(n, ld, generator=g) * 0.3
    r = torch.randn(2, n, generator=g)
    theta = torch.rand(n * (n + 1) // 2, generator=g)
    theta[::9] = -0.5
    u, v = ub[:, :k], vb[:, :k]
    ud, vd, rd = u.double(), v.double(), r.double().sum(0)
    mfull = ud @ vd.t() + vd @ ud.t() + rd[:, None] + rd[None, :]
    iu = torch.triu_indices(n, n)
    ref = mfull[iu[0], iu[1]]
    ref[iu[0] == iu[1]] = 0.0
    ref[(theta.double() < 0) | (theta.double() > 1)] = 0.0
    base = torch.randn(n * (n + 1) // 2, generator=g)
    grad = base.clone().to(device)
    th = theta.clone().to(device)
    lr = 0.05
    scal = torch.zeros(32, dtype=torch.uint8, device=device)
    scal[16:24].view(torch.float64).fill_(lr)
    ub_, vb_, r_ = ub.to(device), vb.to(device), r.to(device)
    prev = ops.theta_grad_form(form)
    try:
        nat.call("lds_theta_grad_ex", nat.ptr(ub_), nat.ptr(vb_), ld, k, nat.ptr(r_), 1, n, 2, nat.ptr(th), n,
                 nat.ptr(grad), mode, nat.ptr(scal), 1.0, ops.form_code(), nat.stream_of(th.device))
        torch.cuda.synchronize()
    finally:
        assert ops.theta_grad_form(prev) == form
    tol = 1e-5 * max(float(ref.abs().max()), 1.0)
    got = grad.cpu().double()
    if mode == 1:
        got = got - base.double()
    elif mode == 3:
        ref = ref + base.double()
        ref[(theta.double() < 0) | (theta.double() > 1)] = 0.0
        ref[iu[0] == iu[1]] = 0.0  # mode 3 writes g (0 on the diagonal), not grad + g
    assert float((got - ref).abs().max()) < tol
    if mode >= 2:
        want = (theta.double() - lr * ref).clamp(0, 1)
        assert float((th.cpu().double() - want).abs().max()) < 1e-5


@pytest.mark.parametrize("form", ["bf16x3", "bf16x3-t64k16-grouped", "bf16x3-t128-grouped", "bf16x3-t128-grouped-i64"])
@pytest.mark.parametrize("n,k,mode", [(300, 264, 2), (2708, 264, 0), (700, 40, 3), (130, 8, 1)])
def test_theta_grad_planes_bit_exact_vs_fp32_operands(device, form, n, k, mode):
    """lds_theta_grad_planes on the split planes of U, V (lds_split_planes,
    the words the engine's factor producers write) gives the same bits as
    lds_theta_grad_ex on the fp32 operands: the split moves out of the kernel,
    the arithmetic does not change."""
    g = torch.Generator().manual_seed(n + k + mode)
    ld = (k + 15) // 16 * 16 + 16
    u = torch.randn(n, ld, generator=g).to(device)
    v = (torch.randn(n, ld, generator=g) * 0.3).to(device)
    r = torch.randn(2, n, generator=g).to(device)
    theta = torch.rand(n * (n + 1) // 2, generator=g)
    theta[::9] = -0.5
    base = torch.randn(n * (n + 1) // 2, generator=g)
    scal = torch.zeros(32, dtype=torch.uint8, device=device)
    scal[16:24].view(torch.float64).fill_(0.05)
    st = nat.stream_of(torch.device(device))
    up = torch.zeros(((ld + 15) // 16) * n * 48, dtype=torch.int16, device=device)
    vp = torch.zeros_like(up)
    nat.call("lds_split_planes", nat.ptr(u), n, ld, ld, nat.ptr(up), st)
    nat.call("lds_split_planes", nat.ptr(v), n, ld, ld, nat.ptr(vp), st)
    outs = []
    prev = ops.theta_grad_form(form)
    try:
        for planes in (False, True):
            th = theta.clone().to(device)
            grad = base.clone().to(device)
            if planes:
                nat.call("lds_theta_grad_planes", nat.ptr(up), nat.ptr(vp), ld, k, nat.ptr(r), 1, n, 2,
                         nat.ptr(th), n, nat.ptr(grad), mode, nat.ptr(scal), 1.0, ops.form_code(), st)
            else:
                nat.call("lds_theta_grad_ex", nat.ptr(u), nat.ptr(v), ld, k, nat.ptr(r), 1, n, 2, nat.ptr(th), n,
                         nat.ptr(grad), mode, nat.ptr(scal), 1.0, ops.form_code(), st)
            torch.cuda.synchronize()
            outs.append((th.cpu(), grad.cpu()))
    finally:
        ops.theta_grad_form(prev)
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


def test_theta_grad_form_default_and_errors(device):
    assert ops.theta_grad_form() == "bf16x3"
    u = torch.zeros((16, 8), device=device)
    g = torch.zeros(16 * 17 // 2, device=device)
    with pytest.raises(nat.NativeError):
        nat.call("lds_theta_grad", nat.ptr(u), nat.ptr(u), 8, 8, 0, 0, 0, 0, 16, nat.ptr(g), 0, 11,
                 nat.stream_of(torch.device(device)))


@pytest.mark.parametrize("n,k,mode", [(2708, 264, 2), (2708, 264, 3), (700, 40, 0), (130, 8, 1), (300, 24, 2),
                                      (257, 48, 1), (3327, 1056, 0)])
def test_theta_grad_pipe_bit_exact(device, n, k, mode):
    """Form 8 (the double-buffered 128-tile) stages the same chunks into the
    same LDS rows and runs the same MFMA order as form 5: identical bits, for
    odd and even chunk counts (k = 264: 17 chunks; 24: 2; 8: 1) and partial
    tiles, in every mode."""
    g = torch.Generator().manual_seed(5 * n + k + mode)
    ld = k + 8
    u = torch.randn(n, ld, generator=g).to(device)
    v = (torch.randn(n, ld, generator=g) * 0.3).to(device)
    r = torch.randn(2, n, generator=g).to(device)
    theta = torch.rand(n * (n + 1) // 2, generator=g)
    theta[::9] = -0.5
    base = torch.randn(n * (n + 1) // 2, generator=g)
    scal = torch.zeros(32, dtype=torch.uint8, device=device)
    scal[16:24].view(torch.float64).fill_(0.05)
    st = nat.stream_of(torch.device(device))
    outs = []
    for form in ("bf16x3-t128-grouped", "bf16x3-t128-pipe", "bf16x3-t128-w8"):
        prev = ops.theta_grad_form(form)
        try:
            th = theta.clone().to(device)
            grad = base.clone().to(device)
            nat.call("lds_theta_grad_ex", nat.ptr(u), nat.ptr(v), ld, k, nat.ptr(r), 1, n, 2, nat.ptr(th), n,
                     nat.ptr(grad), mode, nat.ptr(scal), 1.0, ops.form_code(), st)
            torch.cuda.synchronize()
            outs.append((th.cpu(), grad.cpu()))
        finally:
            ops.theta_grad_form(prev)
    for o in outs[1:]:
        assert torch.equal(outs[0][0], o[0])
        assert torch.equal(outs[0][1], o[1])


@pytest.mark.parametrize("n,k,mode,cuts", [(700, 40, 0, (0, 384, 700)), (1100, 264, 2, (0, 384, 1100)),
                                           (2708, 264, 2, (0, 384, 768, 1408, 2708)), (300, 24, 0, (0, 128, 256, 300))])
def test_theta_grad_band_equals_full(device, n, k, mode, cuts):
    """lds_theta_grad_band (the band-sharded exchange's assembly): the row
    bands [cuts[b], cuts[b+1]) launched one by one give, on every band, the
    bits of the full 128-tile assembly (dθ in mode 0; θ after the fused SGD +
    clamp in mode 2, outside the bands θ untouched), multi-sample operands
    (R of two samples summed), gscale 1/2."""
    g = torch.Generator().manual_seed(7 * n + k + mode)
    u = torch.randn(n, k, generator=g).to(device)
    v = (torch.randn(n, k, generator=g) * 0.3).to(device)
    r = torch.randn(2, n, generator=g).to(device)
    theta = torch.rand(n * (n + 1) // 2, generator=g)
    theta[::9] = -0.5
    scal = torch.zeros(32, dtype=torch.uint8, device=device)
    scal[16:24].view(torch.float64).fill_(0.05)
    st = nat.stream_of(torch.device(device))
    off = lambda r0: r0 * n - r0 * (r0 - 1) // 2  # noqa: E731  (packed index of row r0's first entry)
    prev = ops.theta_grad_form("bf16x3-t128-grouped")
    try:
        th_full = theta.clone().to(device)
        gr_full = torch.zeros_like(th_full)
        nat.call("lds_theta_grad_ex", nat.ptr(u), nat.ptr(v), k, k, nat.ptr(r), 1, n, 2, nat.ptr(th_full), n,
                 nat.ptr(gr_full), mode, nat.ptr(scal), 0.5, ops.form_code(), st)
    finally:
        ops.theta_grad_form(prev)
    for b in range(len(cuts) - 1):
        r0, r1 = cuts[b], cuts[b + 1]
        th = theta.clone().to(device)
        gr = torch.full_like(th, 7.0)
        nat.call("lds_theta_grad_band", nat.ptr(u), nat.ptr(v), k, k, nat.ptr(r), 1, n, 2, nat.ptr(th), n,
                 nat.ptr(gr), mode, nat.ptr(scal), 0.5, r0, r1, st)
        torch.cuda.synchronize()
        lo, hi = off(r0), off(r1)
        assert torch.equal(gr[lo:hi], gr_full[lo:hi]), b
        assert torch.equal(th[lo:hi], th_full[lo:hi]), b
        assert bool((gr[:lo] == 7.0).all()) and bool((gr[hi:] == 7.0).all()), b  # nothing outside the band
        assert torch.equal(th[:lo], theta[:lo].to(device)) and torch.equal(th[hi:], theta[hi:].to(device)), b


@pytest.mark.parametrize("draw_form", ["bf16x3", "bf16x3-t64k16-grouped", "bf16x3-t128-grouped", "bf16x3-t128-w8"])
@pytest.mark.parametrize("n,k,graphs", [(2708, 264, 6), (300, 40, 3), (130, 8, 1), (700, 24, 2), (1000, 16, 21),
                                        (64, 8, 2), (129, 24, 9)])
def test_theta_grad_sgd_draw_equals_sgd_then_draw(device, n, k, graphs, draw_form):
    """lds_theta_grad_sgd_draw (the θ-grad with SGD + clamp, drawing the next
    window's graphs from the θ it writes; the eight-wave 128-tile form by
    default, the 64-tile form when pinned) against lds_theta_grad_sgd
    followed by single lds_sample_bitmask draws of the updated θ: identical θ,
    identical bit rows (graph g draws counter base + offset + g) and degree
    counts equal to the rows' popcounts."""
    g = torch.Generator().manual_seed(n + k + graphs)
    ld = k + 8
    u = torch.randn(n, ld, generator=g).to(device)
    v = (torch.randn(n, ld, generator=g) * 0.3).to(device)
    r = torch.randn(n, generator=g).to(device)
    theta = (torch.rand(n * (n + 1) // 2, generator=g) * 0.4).to(device)
    scal = torch.zeros(64, dtype=torch.uint8, device=device)
    scal[16:24].view(torch.float64).fill_(0.05)
    st = nat.stream_of(torch.device(device))
    words = nat.lib.lds_bitmask_words(n)
    wsi = nat.lib.lds_sample_ws_ints(n)
    base = torch.tensor([11, 0, 0, 0], dtype=torch.int32, device=device)
    seed, tag, off = 4321, tag_for(TAG_GRAPH, 3), 6
    prev = ops.theta_grad_form("bf16x3-t64k16-grouped")
    try:
        th1 = theta.clone()
        nat.call("lds_theta_grad_sgd", nat.ptr(u), nat.ptr(v), ld, k, nat.ptr(r), 1, 1, nat.ptr(th1), n, 0,
                 nat.ptr(scal), ops.form_code(), st)
    finally:
        ops.theta_grad_form(prev)
    th2 = theta.clone()
    bits = torch.zeros((graphs, n, words), dtype=torch.int64, device=device)
    deg = torch.zeros((graphs, wsi), dtype=torch.int32, device=device)
    prev = ops.theta_grad_form(draw_form)  # the eight-wave 128-tile draw (default) or the 64-tile one
    try:
        nat.call("lds_theta_grad_sgd_draw", nat.ptr(u), nat.ptr(v), ld, k, nat.ptr(r), 1, 1, nat.ptr(th2), n, 0,
                 nat.ptr(scal), seed, tag, nat.ptr(base), off, graphs, nat.ptr(bits), words, nat.ptr(deg), ops.form_code(), st)
        torch.cuda.synchronize()
    finally:
        ops.theta_grad_form(prev)
    assert torch.equal(th1, th2)
    one = torch.empty((n, words), dtype=torch.int64, device=device)
    nb = (n + 63) // 64
    for gi in range(graphs):
        nat.call("lds_sample_bitmask", nat.ptr(th1), n, seed, tag, 11 + off + gi, 0, nat.ptr(one), words, st)
        torch.cuda.synchronize()
        assert torch.equal(bits[gi, :, :nb], one[:, :nb]), gi
        pc = torch.zeros(n, dtype=torch.int64, device=device)
        for w in range(nb):
            x = one[:, w]
            for b in range(64):
                pc += (x >> b) & 1
        assert torch.equal(deg[gi, :n].long(), pc), gi


@pytest.mark.parametrize("n,k", [(2708, 264), (300, 40), (130, 8), (129, 21), (64, 16), (1, 8), (700, 0)])
@pytest.mark.parametrize("mode", [0, 1, 2, 3])
def test_theta_grad_direct_bit_exact(device, n, k, mode):
    """Form 10 (lds_theta_grad_direct: pre-split planes of
    lds_split_planes_t128 staged by direct global -> LDS loads, three stage
    buffers) against the 128-tile form on the fp32 operands: identical θ and
    dθ bits in every mode, ragged k and n (zero-padded tiles and chunks), k = 0
    and n = 1."""
    g = torch.Generator().manual_seed(7 * n + k + mode)
    ld = k + 4
    u = torch.randn(n, ld, generator=g).to(device)
    v = (torch.randn(n, ld, generator=g) * 0.3).to(device)
    r = torch.randn(2, n, generator=g).to(device)
    theta = (torch.rand(n * (n + 1) // 2, generator=g) * 1.2 - 0.1).to(device)
    base = torch.randn(n * (n + 1) // 2, generator=g).to(device)
    scal = torch.zeros(64, dtype=torch.uint8, device=device)
    scal[16:24].view(torch.float64).fill_(0.05)
    st = nat.stream_of(torch.device(device))
    kk = max(k, 1)
    ne = nat.lib.lds_planes_t128_elems(n, kk)
    up = torch.full((ne,), -1, dtype=torch.int16, device=device)  # garbage: every word must be written
    vp = torch.full((ne,), -1, dtype=torch.int16, device=device)
    if k > 0:
        nat.call("lds_split_planes_t128", nat.ptr(u), n, ld, k, nat.ptr(up), st)
        nat.call("lds_split_planes_t128", nat.ptr(v), n, ld, k, nat.ptr(vp), st)
    outs = []
    th = theta.clone()
    grad = base.clone()
    prev = ops.theta_grad_form("bf16x3-t128-grouped")
    try:
        nat.call("lds_theta_grad_ex", nat.ptr(u), nat.ptr(v), ld, k, nat.ptr(r), 1, n, 2, nat.ptr(th), n,
                 nat.ptr(grad), mode, nat.ptr(scal), 0.5, ops.form_code(), st)
    finally:
        ops.theta_grad_form(prev)
    outs.append((th, grad))
    th = theta.clone()
    grad = base.clone()
    nat.call("lds_theta_grad_direct", nat.ptr(up), nat.ptr(vp), k, nat.ptr(r), 1, n, 2, nat.ptr(th), n,
             nat.ptr(grad), mode, nat.ptr(scal), 0.5, 0, 0, 0, 0, 0, 0, 0, 0, st)
    torch.cuda.synchronize()
    outs.append((th, grad))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("n,k,graphs", [(2708, 264, 6), (300, 40, 3), (130, 8, 1), (1000, 16, 21), (129, 24, 9)])
def test_theta_grad_direct_draw_equals_sgd_draw(device, n, k, graphs):
    """Form 10 with the next window's draw in its epilogue against
    lds_theta_grad_sgd_draw (form 9): identical θ, bit rows and degree
    accumulators."""
    g = torch.Generator().manual_seed(n + 3 * k + graphs)
    ld = k + 8
    u = torch.randn(n, ld, generator=g).to(device)
    v = (torch.randn(n, ld, generator=g) * 0.3).to(device)
    r = torch.randn(n, generator=g).to(device)
    theta = (torch.rand(n * (n + 1) // 2, generator=g) * 0.4).to(device)
    scal = torch.zeros(64, dtype=torch.uint8, device=device)
    scal[16:24].view(torch.float64).fill_(0.05)
    st = nat.stream_of(torch.device(device))
    words = nat.lib.lds_bitmask_words(n)
    wsi = nat.lib.lds_sample_ws_ints(n)
    base = torch.tensor([11, 0, 0, 0], dtype=torch.int32, device=device)
    seed, tag, off = 4321, tag_for(TAG_GRAPH, 3), 6
    res = []
    for direct in (False, True):
        th = theta.clone()
        bits = torch.zeros((graphs, n, words), dtype=torch.int64, device=device)
        deg = torch.zeros((graphs, wsi), dtype=torch.int32, device=device)
        if direct:
            ne = nat.lib.lds_planes_t128_elems(n, k)
            up = torch.empty(ne, dtype=torch.int16, device=device)
            vp = torch.empty(ne, dtype=torch.int16, device=device)
            nat.call("lds_split_planes_t128", nat.ptr(u), n, ld, k, nat.ptr(up), st)
            nat.call("lds_split_planes_t128", nat.ptr(v), n, ld, k, nat.ptr(vp), st)
            nat.call("lds_theta_grad_direct", nat.ptr(up), nat.ptr(vp), k, nat.ptr(r), 1, 1, 1, nat.ptr(th), n, 0,
                     2, nat.ptr(scal), 1.0, seed, tag, nat.ptr(base), off, graphs, nat.ptr(bits), words,
                     nat.ptr(deg), st)
        else:
            nat.call("lds_theta_grad_sgd_draw", nat.ptr(u), nat.ptr(v), ld, k, nat.ptr(r), 1, 1, nat.ptr(th), n, 0,
                     nat.ptr(scal), seed, tag, nat.ptr(base), off, graphs, nat.ptr(bits), words, nat.ptr(deg), 9, st)
        torch.cuda.synchronize()
        res.append((th, bits, deg))
    for other in res[1:]:
        for a, b in zip(res[0], other):
            assert torch.equal(a, b)


def _spmm_dense(graph_rp, graph_col, s, n, z, ldz=16, out=None, ldy=16, beta=0, grid=0, expect_err=0, checked=True):
    """lds_spmm_norm_dense into `out` (or a new n × 16); the checked form
    (an error word) must read `expect_err` afterwards; checked=False runs the
    unchecked form (err = NULL: canonical columns promised)."""
    dev = z.device
    ws = torch.full((int(nat.lib.lds_spmm_dense_ws_bytes(n)),), 0x5A, dtype=torch.uint8, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    y = out if out is not None else torch.empty(n, ldy, device=dev)
    nat.call("lds_spmm_norm_dense", nat.ptr(graph_rp), nat.ptr(graph_col), nat.ptr(s), n, nat.ptr(z), ldz,
             nat.ptr(y), ldy, beta, nat.ptr(ws), grid, 1, nat.ptr(err) if checked else 0, nat.stream_of(dev))
    torch.cuda.synchronize()
    assert int(err.item()) == expect_err, (int(err.item()), expect_err)
    return y


def _csr_of_dense(a):
    rows, cols = a.nonzero(as_tuple=True)
    rp = torch.zeros(a.size(0) + 1, dtype=torch.int64)
    rp[1:] = torch.cumsum(a.sum(1), 0)
    return rp, cols.int()


@pytest.mark.parametrize("n,high,grid", [(1, 1.0, 0), (17, 1.0, 0), (700, 1.0, 0), (1500, 1.0, 3), (1500, 1.0, -3),
                                         (2600, 0.5, 0), (3000, 0.02, 0), (3001, 1.0, 7), (3001, 1.0, -7),
                                         (3001, 1.0, 40)])
def test_spmm_dense_csr_vs_bitmask_and_fp64(device, n, high, grid):
    """lds_spmm_norm_dense (CSR streamed into LDS bit rows, int8 matrix-core
    product) vs the dense fp64 product, the bitmask aggregation (same digits:
    identical bits where that takes one split) and the other product kernel
    (spill-pass at grid >= 0, the tile kernel at grid < 0: identical bits,
    exact integer sums): ragged n, dense and sparse rows (the sparse fallback
    of the bit setting), grids that force the most rows per block or a
    persistent grid smaller than the tile count (the tile kernel), columns of
    extreme scale; the error word stays 0 on the sampler's canonical CSR.
    Per-column tolerance 1e-5 of max_i Σ_k |Â_ik z_kf|."""
    g = torch.Generator().manual_seed(n + 29)
    theta = torch.rand(n * (n + 1) // 2, generator=g) * high
    graph = ops.sample_graph_from_triu(theta.to(device), n, generator=Generator(n + 1), track_grad=False)
    z = torch.randn(n, 16, generator=g)
    z[:, 3] *= 1e-30
    z[:, 7] *= 1e30
    z[:, 11] = 0.0
    z[: n // 2, 13] *= 1e6
    zd = z.to(device)
    y = _spmm_dense(graph.row_ptr, graph.col, graph.s, n, zd, grid=grid).cpu().double()
    y_other = _spmm_dense(graph.row_ptr, graph.col, graph.s, n, zd, grid=0 if grid < 0 else -256).cpu().double()
    assert torch.equal(y, y_other)
    y_unchecked = _spmm_dense(graph.row_ptr, graph.col, graph.s, n, zd, grid=max(grid, 0), checked=False)
    assert torch.equal(y_unchecked.cpu().double(), y if grid >= 0 else y_other)
    a = graph.normalized_dense().cpu().double()
    ref = a @ z.double()
    scale = (a.abs() @ z.double().abs()).max(0).values.clamp(min=1e-300)
    assert float(((y - ref).abs().max(0).values / scale).max()) < RTOL
    assert torch.all(y[:, 11] == 0)
    y_bit = graph.spmm_bitmask(zd).cpu().double()
    if nat.lib.lds_bitmask_agg_splits(n) == 1:
        assert torch.equal(y, y_bit)
    assert float(((y - y_bit).abs().max(0).values / scale).max()) < RTOL
    # beta = 1 into a strided Y from a strided Z
    zs = torch.zeros(n, 24, device=device)
    zs[:, :16] = zd
    out = torch.ones(n, 20, device=device)
    _spmm_dense(graph.row_ptr, graph.col, graph.s, n, zs, ldz=24, out=out, ldy=20, beta=1, grid=grid)
    o = out.cpu().double()
    assert float(((o[:, :16] - ref - 1.0).abs().max(0).values / scale.clamp(min=1.0)).max()) < RTOL
    assert torch.all(o[:, 16:] == 1.0)


def test_spmm_dense_empty_rows_and_unsorted_columns(device):
    """A general 0/1 CSR with rows in any column order (the bits are set by
    OR), empty rows, long rows straddling the 512-entry steps.  The tile
    kernel (grid < 0) accepts any order; the spill-pass kernel (grid >= 0)
    places every column exactly when its geometry has one column pass, as
    here (n = 1300: three chunks in one pass), so both give the sums of the
    same CSR with its rows sorted, bit for bit, 0 for the empty rows, and no
    error.  (Several passes: test_spmm_dense_unsorted_columns_flag_or_exact.)"""
    n = 1300
    g = torch.Generator().manual_seed(5)
    a = (torch.rand(n, n, generator=g) < 0.45)
    a[7] = False
    a[500:520] = False
    a[n - 1] = False
    rp, col_sorted = _csr_of_dense(a)
    col = col_sorted.clone()
    for i in (3, 900):  # reverse two rows' column order
        b, e = int(rp[i]), int(rp[i + 1])
        col[b:e] = col[b:e].flip(0)
    for i in (11, 1200):  # shuffle two rows (groups of eight whose ends lie close but whose middles do not)
        b, e = int(rp[i]), int(rp[i + 1])
        col[b:e] = col[b:e][torch.randperm(e - b, generator=g)]
    b = int(rp[40])  # one group: ends ascending and one word apart, a middle entry far away
    seg = col[b:b + 8].clone()
    far = int(col[int(rp[41]) - 1])
    col[b + 3] = far
    col[int(rp[41]) - 1] = seg[3]
    s = torch.rand(n, generator=g) + 0.5
    z = torch.randn(n, 16, generator=g)
    ref = s.double()[:, None] * (a.double() @ (s.double()[:, None] * z.double()))
    scale = (a.double() @ (s.double()[:, None] * z.double()).abs()).max(0).values * s.max()
    rpd, cold, sd, zd = rp.int().to(device), col.to(device), s.to(device), z.to(device)
    y_sorted = _spmm_dense(rpd, col_sorted.to(device), sd, n, zd, grid=0).cpu().double()
    ys = []
    for grid in (-256, 0):  # the tile kernel; the spill-pass kernel in one pass
        y = _spmm_dense(rpd, cold, sd, n, zd, grid=grid).cpu().double()
        assert float(((y - ref).abs().max(0).values / scale).max()) < RTOL, grid
        assert torch.all(y[7] == 0) and torch.all(y[500:520] == 0) and torch.all(y[n - 1] == 0), grid
        assert torch.equal(y, y_sorted), grid
        ys.append(y)


def test_spmm_dense_unsorted_columns_flag_or_exact(device):
    """The spill-pass kernel with several column passes (n = 9000, grid 94:
    96-row blocks, three passes of six chunks) on CSRs whose rows are out of
    order: every
    call either gives exactly the sums of the sorted CSR with the error word
    0, or sets LDS_DEVERR_CSR_COLUMNS — never a silent wrong result.  Reversed
    and shuffled rows must be flagged (their first entries belong to the last
    pass); swaps of neighbouring entries inside a lane's 64-column window are
    placed exactly.  A column >= n is flagged too.  The host wrapper
    (CsrGraph.spmm) raises DeviceError on the flag."""
    n, grid = 9000, 94
    g = torch.Generator().manual_seed(17)
    a = torch.rand(n, n, generator=g) < 0.3
    rp, col_sorted = _csr_of_dense(a)
    del a
    s = torch.rand(n, generator=g) + 0.5
    z = torch.randn(n, 16, generator=g)
    rpd, sd, zd = rp.int().to(device), s.to(device), z.to(device)
    y_sorted = _spmm_dense(rpd, col_sorted.to(device), sd, n, zd, grid=grid).cpu()

    def run(col):
        y = torch.empty(n, 16, device=device)
        ws = torch.empty(int(nat.lib.lds_spmm_dense_ws_bytes(n)), dtype=torch.uint8, device=device)
        err = torch.zeros(1, dtype=torch.int32, device=device)
        nat.call("lds_spmm_norm_dense", nat.ptr(rpd), nat.ptr(col.to(device)), nat.ptr(sd), n, nat.ptr(zd), 16,
                 nat.ptr(y), 16, 0, nat.ptr(ws), grid, 1, nat.ptr(err), nat.stream_of(device))
        torch.cuda.synchronize()
        return int(err.item()), y.cpu()

    def row(c, i):
        return slice(int(rp[i]), int(rp[i + 1]))

    cases = {}
    col = col_sorted.clone()  # one reversed row
    col[row(col, 2500)] = col[row(col, 2500)].flip(0)
    cases["reversed"] = (col, True)
    col = col_sorted.clone()  # shuffled rows
    for i in (0, 95, 96, n - 1):
        r = row(col, i)
        col[r] = col[r][torch.randperm(r.stop - r.start, generator=g)]
    cases["shuffled"] = (col, True)
    col = col_sorted.clone()  # the last entry (pass 3) moved to the row's front: re-streamed in pass 2
    r = row(col, 1234)
    col[r] = torch.cat([col[r][-1:], col[r][:-1]])
    cases["last_first"] = (col, True)
    col = col_sorted.clone()  # an entry of the next pass moved to the front: spilled there exactly
    r = row(col, 4321)
    k = int((col[r] >= 3072).nonzero()[0])  # the row's first entry of pass 2
    col[r] = torch.cat([col[r][k:k + 1], col[r][:k], col[r][k + 1:]])
    cases["next_pass_first"] = (col, False)
    col = col_sorted.clone()  # swaps of neighbours (within one lane's eight entries) all over
    for i in range(0, n, 37):
        r = row(col, i)
        k = r.start + 3
        col[k], col[k + 1] = col[k + 1].clone(), col[k].clone()
    cases["neighbour_swaps"] = (col, None)
    col = col_sorted.clone()  # a column past n
    col[int(rp[4000 + 1]) - 1] = n + 5
    cases["past_n"] = (col, True)
    for name, (c, must_flag) in cases.items():
        word, y = run(c)
        assert word in (0, nat.DEVERR_CSR_COLUMNS), (name, word)
        if must_flag is not None:
            assert word == (nat.DEVERR_CSR_COLUMNS if must_flag else 0), name
        if word == 0:
            assert torch.equal(y, y_sorted), name
    # the drop-in wrapper raises on the flag
    graph = ops.CsrGraph(n, rpd, cases["past_n"][0].to(device), sd, (rpd[1:] - rpd[:-1]).int())
    with pytest.raises(nat.DeviceError, match="lds_spmm_norm_dense"):
        graph.spmm(zd)


@pytest.mark.parametrize("grid", [0, 63])
def test_spmm_dense_spill_pass_row_shapes(device, grid):
    """The spill-pass kernel (the product at grid >= 0; ascending columns) on
    rows that take each of its paths, against the tile kernel (grid < 0, any
    column order; identical bits: exact integer sums) and fp64: rows whose
    entries crowd the first columns (the stream stops at the predicted pass
    end before the pass boundary and the row is finished with blocking
    loads), rows crowding the last columns (every step of the early passes
    lies past pass p + 1: re-read later), sparse rows whose steps span
    several passes, empty rows, full rows, and a last row that ends the array
    off a 16-byte boundary; no error on these canonical rows.  grid 63 gives
    96-row blocks and two passes of six chunks at n = 6000.  (The round-4 variants of the
    kernel: tests/test_spmm_variants_gpu.py.)"""
    n = 6000
    g = torch.Generator().manual_seed(11)
    dens = torch.rand(n, generator=g) * 0.6
    a = torch.rand(n, n, generator=g) < dens[:, None]
    a[0:40, 1000:] = False          # crowd the first columns
    a[40:80, :4500] = False         # crowd the last columns
    a[80:120] = torch.rand(40, n, generator=g) < 0.002   # sparse: steps span passes
    a[120] = False
    a[121] = True
    a[200:260:3] = False
    a[n - 1] = False
    a[n - 1, 5] = True
    a[n - 1, 7] = True
    a[n - 1, 5999] = True           # nnz off a multiple of four (checked below)
    rp, col = _csr_of_dense(a)
    if int(rp[-1]) % 4 == 0:
        a[n - 2, 3] = not bool(a[n - 2, 3])
        rp, col = _csr_of_dense(a)
    assert int(rp[-1]) % 4 != 0
    s = torch.rand(n, generator=g) + 0.5
    z = torch.randn(n, 16, generator=g)
    rpd, cold, sd, zd = rp.int().to(device), col.to(device), s.to(device), z.to(device)
    y = _spmm_dense(rpd, cold, sd, n, zd, grid=grid)  # the product (spill-pass kernel), checked
    y_tile = _spmm_dense(rpd, cold, sd, n, zd, grid=-256)
    assert torch.equal(y.cpu(), y_tile.cpu())
    assert torch.equal(_spmm_dense(rpd, cold, sd, n, zd, grid=grid, checked=False).cpu(), y.cpu())  # unchecked
    ad = a.double()
    ref = s.double()[:, None] * (ad @ (s.double()[:, None] * z.double()))
    scale = (ad @ (s.double()[:, None] * z.double()).abs()).max(0).values * s.max()
    assert float(((y.cpu().double() - ref).abs().max(0).values / scale).max()) < RTOL
    assert torch.all(y[120] == 0)


@pytest.mark.parametrize("samples,count,n", [(5, 3, 700), (16, 2, 257)])
def test_batched_draw_sample_ranges_equal_single_draws(device, samples, count, n):
    """The window draw with replica samples split over grid.z (sample ranges
    per block; at these sizes every sample gets its own block range) against
    one single draw per (graph, sample) with that sample's tag: identical
    bits, and degree counts equal to the rows' popcounts (the fused CSR path
    the engine uses)."""
    g = torch.Generator(device=device).manual_seed(n + samples)
    theta = torch.rand(n * (n + 1) // 2, generator=g, device=device)
    words = nat.lib.lds_bitmask_words(n)
    wsi = nat.lib.lds_sample_ws_ints(n)
    st = nat.stream_of(device)
    base = torch.tensor([5, 0, 0, 0], dtype=torch.int32, device=device)
    G = count * samples
    bits = torch.empty((count, samples, n, words), dtype=torch.int64, device=device)
    deg = torch.empty((count, samples, wsi), dtype=torch.int32, device=device)
    row_ptr = torch.empty((G, n + 1), dtype=torch.int32, device=device)
    col = torch.empty((G, n * n), dtype=torch.int32, device=device)
    s = torch.empty((G, n), dtype=torch.float32, device=device)
    ell = torch.empty((G, n * 2 * 64), dtype=torch.int32, device=device)
    seed, tag, off = 77, tag_for(TAG_GRAPH, 0), 2
    nat.call("lds_sample_graphs_multi", nat.ptr(theta), n, seed, tag, 1, nat.ptr(base), off, count, samples,
             nat.ptr(bits), words, nat.ptr(deg), nat.ptr(row_ptr), nat.ptr(col), n * n, nat.ptr(s), nat.ptr(ell),
             0, 0, 0, st)
    one = torch.empty((n, words), dtype=torch.int64, device=device)
    nb = (n + 63) // 64
    for gi in range(count):
        for z in range(samples):
            nat.call("lds_sample_bitmask", nat.ptr(theta), n, seed, tag + z, 5 + off + gi, 0, nat.ptr(one), words,
                     st)
            assert torch.equal(bits[gi, z, :, :nb], one[:, :nb]), (gi, z)
            pc = torch.zeros(n, dtype=torch.int64, device=device)
            for w in range(nb):  # popcount per row, word by word
                x = one[:, w]
                for b in range(64):
                    pc += (x >> b) & 1
            assert torch.equal(deg[gi, z, :n].long(), pc), (gi, z)
