"""Torch-facing hot-path ops over the C-ABI library, with autograd.

Graphs never exist as dense N×N matrices here.  A sampled graph is a
`SampledGraph`: the symmetric bit matrix + CSR (self-loops included) +
s = deg^-1/2 on device, plus a back-link to θ for the hypergradient.

Gradients w.r.t. θ are low-rank.  Each aggregation Y = ÂZ of a graph
contributes dL/dÂ = G Zᵀ (G = dL/dY), and the θ-gradient of the whole graph is
a rank-2k symmetric update of the packed triangle (lds_theta_grad).  To get
there through PyTorch autograd — including the create_graph inner steps and
the double backward of the hyper step — every graph carries a small "token"
tensor (n × width, produced from θ by _GraphToken).  Each aggregation that
uses the graph reserves its own columns ("slot") of the token; its backward
returns the slot factors [s⊙G | s⊙Z | r] in those columns and zeros elsewhere,
so autograd's sum over uses concatenates the factors.  _GraphToken.backward
then assembles dθ once per graph.  A is differentiated once, so the factors
never need their own gradient ("closure of the kernel set").
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Tuple

import torch
from torch.autograd import Function

from . import _native as nat
from .rng import TAG_DROP_H, TAG_DROP_X, Generator, default_generator

_FULL_CAPACITY_LIMIT = 1 << 26  # col buffer upper bound n*n below this many entries

TOKEN_KCAP = 64  # U and V columns per token chunk (4 slots of 16 features)
TOKEN_RCAP = 8   # r columns per token chunk


def _stream(t: torch.Tensor) -> int:
    return nat.stream_of(t.device)


def _f32c(t: torch.Tensor, what: str) -> torch.Tensor:
    nat.require_device(t, what)
    if t.dtype != torch.float32:
        raise TypeError(f"ldsgnn {what}: expected float32, got {t.dtype}")
    if t.dim() == 2 and t.stride(1) == 1 and t.stride(0) >= t.size(1):
        return t
    return t.contiguous()


# ---------------------------------------------------------------------------
# graph containers
# ---------------------------------------------------------------------------


class CsrGraph:
    """A normalised graph on device: Â = diag(s)·Ã·diag(s) in CSR form.

    `row_ptr` (n+1, int32), `col` (>= nnz, int32, ascending per row, self-loop
    included), `s` (n, fp32), `deg` (n, int32), optional `bits` (n × words
    uint64 stored as int64) — the layouts of include/ldsgnn.h.
    """

    # columns ascending and distinct in [0, n) by construction (set by the
    # library's own samplers / fills; a caller-built CSR is checked)
    canonical_columns = False

    def __init__(self, n: int, row_ptr: torch.Tensor, col: torch.Tensor, s: torch.Tensor,
                 deg: torch.Tensor, bits: Optional[torch.Tensor] = None):
        self.n = n
        self.row_ptr, self.col, self.s, self.deg, self.bits = row_ptr, col, s, deg, bits
        self._nnz: Optional[int] = None

    # tensor-like surface used by the reference API (is_square_matrix etc.)
    @property
    def shape(self) -> torch.Size:
        return torch.Size((self.n, self.n))

    def size(self, dim: Optional[int] = None):
        return self.shape if dim is None else self.n

    def dim(self) -> int:
        return 2

    @property
    def device(self) -> torch.device:
        return self.row_ptr.device

    @property
    def requires_grad(self) -> bool:
        return False

    def nnz(self) -> int:
        """Stored entries incl. self-loops (host sync on first call)."""
        if self._nnz is None:
            self._nnz = int(self.row_ptr[self.n].item())
        return self._nnz

    def num_edges(self) -> int:
        """Undirected off-diagonal edges."""
        return (self.nnz() - self.n) // 2

    # mean entries per row from which the column-blocked LDS kernel
    # (lds_spmm_norm_blocked) replaces the row-group kernel (F = 16 only)
    LONG_ROW_DEGREE = 256

    def long_rows(self) -> bool:
        return self.n >= 1024 and self.nnz() >= self.LONG_ROW_DEGREE * self.n

    def _block_ptr(self) -> torch.Tensor:
        bp = getattr(self, "_bptr", None)
        if bp is None:
            nb = nat.lib.lds_spmm_block_count(self.n)
            bp = torch.empty(self.n * (nb + 1), dtype=torch.int32, device=self.device)
            nat.call("lds_csr_block_ptr", nat.ptr(self.row_ptr), nat.ptr(self.col), self.n, nat.ptr(bp),
                     _stream(self.s))
            self._bptr = bp
        return bp

    def spmm(self, z: torch.Tensor, out: Optional[torch.Tensor] = None, beta: int = 0,
             blocked: Optional[bool] = None) -> torch.Tensor:
        """Y = Â·Z; no autograd.  Row-group kernel (lds_spmm_norm), or for long
        rows at F = 16 the CSR spill-pass kernel on the int8 matrix cores
        (lds_spmm_norm_dense; 165-168 against 414 µs for the column-blocked kernel
        at BASELINE config 5; needs the ascending columns this class holds: a
        CSR whose column order the kernel cannot aggregate faithfully raises
        ldsgnn._native.DeviceError on the graph's first call).  `blocked=True` forces the column-blocked kernel
        (lds_spmm_norm_blocked), `blocked=False` the row-group kernel."""
        z = _f32c(z, "spmm")
        if z.dim() != 2 or z.size(0) != self.n:
            raise ValueError(f"spmm: Z must be {self.n}×F, got {tuple(z.shape)}")
        f = z.size(1)
        if out is None:
            out = torch.empty((self.n, f), dtype=torch.float32, device=z.device)
        if blocked is None and f == 16 and self.long_rows() and self.n <= nat.lib.lds_spmm_dense_max_n() \
                and self.col.data_ptr() % 16 == 0:
            ws = getattr(self, "_dense_ws", None)
            if ws is None:
                ws = torch.empty(int(nat.lib.lds_spmm_dense_ws_bytes(self.n)), dtype=torch.uint8, device=z.device)
                self._dense_ws = ws
                self._dense_err = torch.zeros(1, dtype=torch.int32, device=z.device)
            # a graph this library sampled has canonical columns (the unchecked
            # form); any other CSR runs the checked form, which flags a column
            # order it cannot aggregate faithfully (a property of the CSR:
            # read on the graph's first call, one sync)
            checked = not self.canonical_columns
            if checked and not getattr(self, "_dense_checked", False) and torch.cuda.is_current_stream_capturing():
                # the check's error word is read on the host; inside a capture it
                # never would be, so a wrong column order would give wrong sums
                # silently on every replay (round-5 ADVICE): verify eagerly first
                raise RuntimeError("CsrGraph.spmm: the column order of this CSR has not been checked yet; run one "
                                   "eager spmm on it before capturing (canonical_columns=False graphs are checked "
                                   "once, on the host)")
            nat.call("lds_spmm_norm_dense", nat.ptr(self.row_ptr), nat.ptr(self.col), nat.ptr(self.s), self.n,
                     nat.ptr(z), z.stride(0), nat.ptr(out), out.stride(0), beta, nat.ptr(ws), 0, 1,
                     nat.ptr(self._dense_err) if checked else 0, _stream(z))
            if checked and not getattr(self, "_dense_checked", False) and \
                    not torch.cuda.is_current_stream_capturing():
                word = int(self._dense_err.item())
                if word:
                    self._dense_err.zero_()
                    nat.raise_device_error(word, "CsrGraph.spmm (lds_spmm_norm_dense)")
                self._dense_checked = True
            return out
        use_blocked = (f == 16 and self.long_rows()) if blocked is None else blocked
        if use_blocked:
            if f != 16 or z.stride(0) % 4 or z.data_ptr() % 16:
                raise ValueError("blocked spmm: F = 16, 16-byte aligned rows")
            nb = nat.lib.lds_spmm_block_count(self.n)
            part = torch.empty((nb, self.n, 16), dtype=torch.float32, device=z.device)
            nat.call("lds_spmm_norm_blocked", nat.ptr(self._block_ptr()), nat.ptr(self.col), nat.ptr(self.s),
                     self.n, nat.ptr(z), z.stride(0), nat.ptr(out), out.stride(0), beta, nat.ptr(part), _stream(z))
            return out
        nat.call("lds_spmm_norm", nat.ptr(self.row_ptr), nat.ptr(self.col), nat.ptr(self.s), self.n,
                 nat.ptr(z), f, z.stride(0), nat.ptr(out), out.stride(0), beta, _stream(z))
        return out

    def spmm_bitmask(self, z: torch.Tensor, out: Optional[torch.Tensor] = None, beta: int = 0) -> torch.Tensor:
        """Y = Â·Z from the sampled bitmask on the int8 matrix cores
        (lds_aggregate_bitmask; F = 16; dense graphs).  Needs `bits`."""
        if self.bits is None:
            raise ValueError("spmm_bitmask: this graph carries no bitmask")
        z = _f32c(z, "spmm_bitmask")
        if z.dim() != 2 or z.size(0) != self.n or z.size(1) != 16:
            raise ValueError(f"spmm_bitmask: Z must be {self.n}×16, got {tuple(z.shape)}")
        if out is None:
            out = torch.empty((self.n, 16), dtype=torch.float32, device=z.device)
        ws = torch.empty(int(nat.lib.lds_bitmask_agg_ws_bytes(self.n)), dtype=torch.uint8, device=z.device)
        nat.call("lds_aggregate_bitmask", nat.ptr(self.bits), self.bits.size(1), nat.ptr(self.s), self.n, nat.ptr(z),
                 z.stride(0), nat.ptr(out), out.stride(0), beta, nat.ptr(ws), _stream(z))
        return out

    def to_dense(self) -> torch.Tensor:
        """Ã as a dense 0/1 matrix (diagonal = 1).  Inspection only."""
        n = self.n
        rp = self.row_ptr.long()
        counts = rp[1:] - rp[:-1]
        rows = torch.repeat_interleave(torch.arange(n, device=self.device), counts)
        cols = self.col[: int(rp[-1].item())].long()
        a = torch.zeros((n, n), dtype=torch.float32, device=self.device)
        a[rows, cols] = 1.0
        return a

    def normalized_dense(self) -> torch.Tensor:
        """Â as a dense matrix.  Inspection only."""
        return self.s[:, None] * self.to_dense() * self.s[None, :]


class _TokenChunk:
    def __init__(self, graph: "SampledGraph", kcap: int, rcap: int):
        self.graph = graph
        self.kcap, self.rcap = kcap, rcap
        self.kused = 0
        self.rused = 0
        self.token: Optional[torch.Tensor] = None

    @property
    def width(self) -> int:
        return 2 * self.kcap + self.rcap


class SampledGraph(CsrGraph):
    """A graph drawn from θ.  Gradients flow to θ through the token chunks."""

    canonical_columns = True  # the sampler's fill writes each row's columns ascending

    def __init__(self, n, row_ptr, col, s, deg, bits, theta: Optional[torch.Tensor]):
        super().__init__(n, row_ptr, col, s, deg, bits)
        self.theta = theta
        self._chunks: List[_TokenChunk] = []

    @property
    def requires_grad(self) -> bool:
        return self.theta is not None and self.theta.requires_grad and torch.is_grad_enabled()

    def new_slot(self, f: int) -> Tuple[Optional[torch.Tensor], Optional[Tuple[int, int]]]:
        """Reserve f U/V columns + 1 r column for one aggregation."""
        if not self.requires_grad:
            return None, None
        fpad = (f + 3) & ~3
        ch = self._chunks[-1] if self._chunks else None
        if ch is None or ch.kused + fpad > ch.kcap or ch.rused + 1 > ch.rcap:
            ch = _TokenChunk(self, max(TOKEN_KCAP, fpad), TOKEN_RCAP)
            ch.token = _GraphToken.apply(self.theta, ch)
            self._chunks.append(ch)
        slot = (ch.kused, ch.rused)
        ch.kused += fpad
        ch.rused += 1
        return ch.token, (id(ch), slot[0], slot[1], fpad, ch)


# ---------------------------------------------------------------------------
# sampling
# ---------------------------------------------------------------------------


def sample_graph_from_triu(theta: torch.Tensor, n: int, generator: Optional[Generator] = None,
                           u_inject: Optional[torch.Tensor] = None, track_grad: bool = True,
                           keep: Optional[torch.Tensor] = None) -> SampledGraph:
    """Draw A ~ Bernoulli(clamp(θ, 0, 1)) on the upper triangle, symmetrise, add
    self-loops, build CSR + s (lds_sample_graph).  `u_inject`: n×n uniforms
    replacing the keyed Philox draws (reference-RNG parity mode).  `keep`
    (packed triu, 0/1): sparsification of the SAMPLE (src/models/sampling.py:
    19-44 applied to the Bernoulli draw) — entry (i, j) is drawn as
    u_ij < θ_ij·keep_ij, i.e. exactly sample ⊙ keep with the same uniforms,
    while the straight-through gradient still reaches every θ_ij."""
    nat.require_device(theta, "sample")
    if theta.dim() != 1 or theta.numel() != n * (n + 1) // 2 or theta.dtype != torch.float32:
        raise ValueError("theta must be the float32 packed upper triangle incl. diagonal")
    th = theta.detach()
    if not th.is_contiguous():
        th = th.contiguous()
    if keep is not None:
        if keep.shape != th.shape:
            raise ValueError("keep must be a packed upper-triangle mask like theta")
        th = (th.clamp(0.0, 1.0) * (keep.detach().to(th.device) != 0).to(th.dtype)).contiguous()
    gen = generator or default_generator
    seed, tag, counter = gen.next_graph()
    dev = theta.device
    words = nat.lib.lds_bitmask_words(n)
    bits = torch.empty((n, words), dtype=torch.int64, device=dev)
    deg = torch.empty(n, dtype=torch.int32, device=dev)
    row_ptr = torch.empty(n + 1, dtype=torch.int32, device=dev)
    s = torch.empty(n, dtype=torch.float32, device=dev)
    st = _stream(th)
    if u_inject is not None:
        u_inject = _f32c(u_inject, "sample u_inject")
        if u_inject.shape != (n, n) or not u_inject.is_contiguous():
            raise ValueError("u_inject must be a contiguous n×n float32 tensor")
    nat.call("lds_sample_bitmask", nat.ptr(th), n, seed, tag, counter, nat.ptr(u_inject),
             nat.ptr(bits), words, st)
    nat.call("lds_bitmask_degree", nat.ptr(bits), n, words, nat.ptr(deg), nat.ptr(s), st)
    nat.call("lds_exclusive_scan", nat.ptr(deg), n, nat.ptr(row_ptr), st)
    if n * n <= _FULL_CAPACITY_LIMIT:
        capacity = n * n
    else:  # exact size: one host sync
        capacity = int(row_ptr[n].item())
    col = torch.empty(max(capacity, 1), dtype=torch.int32, device=dev)
    nat.call("lds_bitmask_fill_csr", nat.ptr(bits), n, words, nat.ptr(row_ptr), nat.ptr(col),
             capacity, 0, st)
    return SampledGraph(n, row_ptr, col, s, deg, bits, theta if track_grad else None)


def csr_graph_from_dense(adj: torch.Tensor) -> CsrGraph:
    """A fixed 0/1 adjacency (e.g. the dataset graph, BASELINE config 1) in the
    hot-path layout.  Off-diagonal entries must be 0/1 and symmetric; the
    diagonal is ignored (self-loops are set, src/utils/graph.py:123-133)."""
    nat.require_device(adj, "csr_graph_from_dense")
    n = adj.size(0)
    a = adj.detach().to(torch.float32).clone()
    a.fill_diagonal_(1.0)
    if not bool(((a == 0) | (a == 1)).all()) or not torch.equal(a, a.t()):
        raise ValueError("csr_graph_from_dense needs a symmetric 0/1 adjacency")
    deg = a.sum(1).to(torch.int32)
    row_ptr = torch.zeros(n + 1, dtype=torch.int32, device=adj.device)
    row_ptr[1:] = torch.cumsum(deg, 0).to(torch.int32)
    col = a.nonzero()[:, 1].to(torch.int32).contiguous()  # row-major -> ascending per row
    s = torch.empty(n, dtype=torch.float32, device=adj.device)
    # same correctly-rounded reciprocal(sqrt(d)) as the sampler's degree pass
    nat.call("lds_csr_degree_scale", nat.ptr(row_ptr), n, nat.ptr(deg), nat.ptr(s), _stream(s))
    return CsrGraph(n, row_ptr, col, s, deg, None)


# ---------------------------------------------------------------------------
# autograd functions
# ---------------------------------------------------------------------------


class _GraphToken(Function):
    """θ -> zero token; backward assembles dθ of one graph (lds_theta_grad)."""

    @staticmethod
    def forward(ctx, theta, chunk):
        ctx.chunk = chunk
        ctx.theta = theta.detach()  # clamp mask read at backward time (θ stays in [0,1])
        return torch.zeros((chunk.graph.n, chunk.width), dtype=torch.float32, device=theta.device)

    @staticmethod
    def backward(ctx, dtok):
        ch: _TokenChunk = ctx.chunk
        theta = ctx.theta
        dtok = dtok.contiguous()
        grad = torch.empty_like(theta)
        w = ch.width
        base = dtok.data_ptr()
        nat.call("lds_theta_grad", base, base + 4 * ch.kcap, w, ch.kused, base + 8 * ch.kcap, w,
                 ch.rused, nat.ptr(theta), ch.graph.n, nat.ptr(grad), 0, form_code(), _stream(theta))
        return grad, None


def _write_slot(dtok: torch.Tensor, slot, gy: torch.Tensor, z: torch.Tensor, y: torch.Tensor,
                dz: torch.Tensor, s: torch.Tensor, n: int) -> None:
    _, koff, roff, fpad, ch = slot
    w = ch.width
    base = dtok.data_ptr()
    f = z.size(1)
    nat.call("lds_slot_factors", nat.ptr(gy), gy.stride(0), nat.ptr(z), z.stride(0), nat.ptr(y),
             y.stride(0), nat.ptr(dz), dz.stride(0), nat.ptr(s), n, f, fpad,
             base + 4 * koff, w, base + 4 * (ch.kcap + koff), w, base + 4 * (2 * ch.kcap + roff), w,
             _stream(dtok))


class _Aggregate(Function):
    """Y = Â·Z.  Backward: dZ = Â·G (recorded when create_graph), token slot."""

    @staticmethod
    def forward(ctx, z, token, graph, slot):
        z = _f32c(z, "aggregate")
        y = graph.spmm(z)
        ctx.graph, ctx.slot = graph, slot
        ctx.save_for_backward(z, y, token)
        return y

    @staticmethod
    def backward(ctx, gy):
        z, y, token = ctx.saved_tensors
        graph, slot = ctx.graph, ctx.slot
        need_z, need_tok = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        gy = _f32c(gy, "aggregate backward")
        dz = None
        if need_z or need_tok:
            if need_z and torch.is_grad_enabled():
                dz = aggregate(gy, graph)  # create_graph: a differentiable use of the graph
            else:
                dz = graph.spmm(gy)
        dtok = None
        if need_tok:
            dtok = torch.zeros_like(token)
            with torch.no_grad():
                _write_slot(dtok, slot, gy, z, y, dz.detach(), graph.s, graph.n)
        return (dz if need_z else None), dtok, None, None


def aggregate(z: torch.Tensor, graph: CsrGraph) -> torch.Tensor:
    """Â·Z for a hot-path graph, differentiable in Z and (sampled graphs) θ."""
    if isinstance(graph, SampledGraph) and graph.requires_grad:
        token, slot = graph.new_slot(z.size(1))
        return _Aggregate.apply(z, token, graph, slot)
    if z.requires_grad and torch.is_grad_enabled():
        return _Aggregate.apply(z, None, graph, None)
    return graph.spmm(z)


class _KeyedDropout(Function):
    @staticmethod
    def forward(ctx, x, keep, scale, key):
        ctx.keep, ctx.scale, ctx.key = keep, scale, key
        return _dropout_raw(x, keep, scale, key)

    @staticmethod
    def backward(ctx, gy):
        if torch.is_grad_enabled():
            gx = _KeyedDropout.apply(gy, ctx.keep, ctx.scale, ctx.key)
        else:
            gx = _dropout_raw(gy, ctx.keep, ctx.scale, ctx.key)
        return gx, None, None, None


def _dropout_raw(x: torch.Tensor, keep: float, scale: float, key) -> torch.Tensor:
    x = _f32c(x, "dropout")
    rows, cols = x.shape
    y = torch.empty((rows, cols), dtype=torch.float32, device=x.device)
    seed, tag, counter = key
    nat.call("lds_dropout", nat.ptr(x), x.stride(0), nat.ptr(y), cols, rows, cols, keep, scale, seed,
             tag, counter, _stream(x))
    return y


def keyed_dropout(x: torch.Tensor, p: float, key) -> torch.Tensor:
    """F.dropout with a keyed mask: keep iff u(i, j) < 1 - p, scale 1/(1-p)."""
    import numpy as np
    keep = np.float32(1.0) - np.float32(p)
    scale = np.float32(1.0) / keep
    if x.requires_grad and torch.is_grad_enabled():
        return _KeyedDropout.apply(x, float(keep), float(scale), key)
    return _dropout_raw(x, float(keep), float(scale), key)


# ---------------------------------------------------------------------------
# plain kernels
# ---------------------------------------------------------------------------


def sgd_clamp_(theta: torch.Tensor, grad: torch.Tensor, lr: float) -> torch.Tensor:
    """θ = clamp(θ - lr·grad, 0, 1) in place (lds_sgd_clamp)."""
    nat.require_device(theta, "sgd_clamp")
    if not (theta.is_contiguous() and grad.is_contiguous()) or theta.numel() != grad.numel():
        raise ValueError("sgd_clamp_: contiguous θ and grad of equal size required")
    nat.call("lds_sgd_clamp", nat.ptr(theta), nat.ptr(grad), float(lr), theta.numel(), _stream(theta))
    return theta


def theta_grad(u: torch.Tensor, v: torch.Tensor, r: torch.Tensor, n: int,
               theta: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
               accumulate: bool = False) -> torch.Tensor:
    """Packed-triangle θ-gradient from factors (lds_theta_grad).  u, v: n×k
    (already scaled by s), r: n×nr (summed per row)."""
    u, v = _f32c(u, "theta_grad"), _f32c(v, "theta_grad")
    if u.shape != v.shape or u.stride(0) != v.stride(0):
        raise ValueError("theta_grad: u and v must share shape and row stride")
    r = _f32c(r.reshape(n, -1), "theta_grad")
    if out is None:
        out = torch.empty(n * (n + 1) // 2, dtype=torch.float32, device=u.device)
    nat.call("lds_theta_grad", nat.ptr(u), nat.ptr(v), u.stride(0), u.size(1), nat.ptr(r),
             r.stride(0), r.size(1), nat.ptr(theta), n, nat.ptr(out), int(accumulate), form_code(), _stream(u))
    return out


THETA_GRAD_FORMS = {"fp32": 0, "bf16x3": 1, "bf16x3-t64k16": 2, "bf16x3-t64k32": 3, "bf16x3-t128": 4,
                    "bf16x3-t128-grouped": 5, "bf16x3-t64k16-grouped": 6, "bf16x3-t128-grouped-i64": 7,
                    "bf16x3-t128-pipe": 8, "bf16x3-t128-w8": 9, "bf16x3-direct": 10}


_theta_form = "bf16x3"


def theta_grad_form(form: Optional[str] = None) -> str:
    """Select the default arithmetic form of the θ-gradient assembly that this
    module's callers pass to the C-ABI (every lds_theta_grad* entry point takes
    the form per call; the library keeps no form state): "bf16x3" (default:
    fp32 operands split into three bf16 words, six bf16 MFMAs per product,
    fp32 accuracy; tile shape chosen by problem size), one pinned split-bf16
    variant (64-tiles with 16- or 32-wide k chunks, 128-tiles in plain or
    XCD-grouped order, the pipelined 128-tiles), "bf16x3-direct" (the
    direct-staged eight-wave 128-tile on pre-split planes: an LdsEngine then
    has its factor producers write the planes; entry points on fp32 operands
    run the by-shape form), or "fp32" (fp32-in MFMA).
    Returns the previous default.  An LdsEngine with its own `theta_form`
    ignores this default; HIP graphs keep the form they were captured with."""
    global _theta_form
    prev = _theta_form
    if form is not None:
        if form not in THETA_GRAD_FORMS:
            raise ValueError(f"unknown θ-grad form {form!r}; one of {sorted(THETA_GRAD_FORMS)}")
        _theta_form = form
    return prev


def form_code(form: Optional[str] = None) -> int:
    """The C-ABI `form` argument of `form` (default: theta_grad_form())."""
    return THETA_GRAD_FORMS[_theta_form if form is None else form]


def philox_uniform(seed: int, tag: int, counter: int, rows: int, cols: int,
                   device="cuda") -> torch.Tensor:
    out = torch.empty((rows, cols), dtype=torch.float32, device=device)
    nat.call("lds_philox_uniform", seed, tag, counter, rows, cols, nat.ptr(out), _stream(out))
    return out


__all__ = [
    "CsrGraph", "SampledGraph", "sample_graph_from_triu", "csr_graph_from_dense", "aggregate",
    "keyed_dropout", "sgd_clamp_", "theta_grad", "theta_grad_form", "form_code", "philox_uniform", "TAG_DROP_X", "TAG_DROP_H",
]
