"""Fused LDS engine: the bilevel hot path as hand-written HIP kernels.

What it replaces (LDS configuration of the reference):
  * an inner step — InnerProblemTrainer.train_step (src/trainers/inner.py:55-74):
    sample A ~ θ, GCN forward, NLL on the train mask, create_graph backward,
    higher's differentiable Adam step;
  * a hyper step — OuterProblemTrainer.train_step (src/trainers/outer.py:57-87):
    fresh sample, forward with the current weights, NLL on opt_mask,
    loss.backward through the outer graph and every unrolled inner step since
    the last detach, SGD on θ, StepLR, clamp; then both trainers detach
    (src/trainers/bilevel.py:109-114).

How: autograd is replaced by a hand-derived reverse pass.  Each
inner step records a tape slot (graph CSR + s, 10 n×16 activation arrays,
w/m/v/g' of the Adam step).  The hyper step runs the outer forward/backward,
then walks the tape backwards: Adam reverse → Hessian-vector reverse of the
backward (4 aggregations, 2 X-products, 1 reduction); every aggregation emits
its θ-gradient factor pair, and ONE lds_theta_grad call (rank K = 48 per inner
graph + 24 outer at C = 7) assembles the window's dθ, followed by SGD + clamp
with the device-resident learning rate.  RNG counters, the Adam step and the
learning rate live on the device, so `capture_window()` records a whole
τ-window (τ inner steps + the hyper step) as one HIP graph that replays with
advancing state.

Layout: per-node arrays are n × 16 fp32 (hidden 16; classes padded to 16);
parameters are one flat vector [W0ᵀ (fin×16) | b0 (16) | W1 (C×16) | b1 (C)].

Replica samples (`samples=S`, SURVEY §8(e), BASELINE configs 3/4): S independent
Monte-Carlo chains — own graphs, dropout masks (replica tags replica0 + b), GCN
weights and Adam state — share θ, X and the scalars, and run in the SAME
launches (grid.y = sample; include/ldsgnn.h LdsBatch).  Every per-sample array
carries a leading S dimension.  The hyper step assembles the mean of the S
hypergradients in one rank-(S·K) update (lds_theta_grad_ex, gscale = 1/S);
S = 1 is the reference's single chain.
"""
from __future__ import annotations

import ctypes
from collections import OrderedDict
from typing import List, Optional

import numpy as np

import torch

from . import _native as nat
from .rng import TAG_DROP_H, TAG_DROP_X, TAG_GRAPH, Generator, tag_for

HID = 16
ELL = 64  # entries per row in a graph's ELL head (kEllWidth in csrc/common.hpp)
_RED_LEN = 304
_TAB_MAX = 256  # Adam table entries (kAdamTabMax in engine.hip)
_ACT = ("h0", "y0", "h1d", "h2", "o", "p", "d_o", "dh2", "dy0", "dh0")


class _Graph:
    """Device buffers of one sampled graph per replica sample (CSR with
    self-loops + s): arrays [S, ...]."""

    def __init__(self, n: int, cap: int, dev, views=None, samples: int = 1, bptr_len: int = 0, words: int = 0):
        if views is not None:
            self.row_ptr, self.col, self.s, self.ell, self.bptr, self.bits = views
            return
        S = samples
        self.bits = torch.empty((S, n, words), dtype=torch.int64, device=dev)  # the sampled bitmask
        self.row_ptr = torch.empty((S, n + 1), dtype=torch.int32, device=dev)
        self.col = torch.empty((S, max(cap, 1)), dtype=torch.int32, device=dev)
        self.s = torch.empty((S, n), dtype=torch.float32, device=dev)
        self.ell = torch.empty((S, n * 2 * ELL), dtype=torch.int32, device=dev)  # ELL head {j, s_j}
        # long rows: segment starts per (row, column block) for lds_spmm_norm_blocked
        self.bptr = torch.empty((S, bptr_len), dtype=torch.int32, device=dev) if bptr_len else None


class _GraphBatch:
    """Contiguous storage for the τ+1 graphs of a window, so that one batched
    lds_sample_graphs launch set draws them all (θ is fixed within a window)."""

    def __init__(self, count: int, n: int, words: int, cap: int, dev, samples: int = 1, bptr_len: int = 0):
        self.count, self.cap = count, cap
        S = samples
        self.bits = torch.empty((count, S, n, words), dtype=torch.int64, device=dev)
        # sampler workspace (degrees + row-block totals, lds_sample_ws_ints):
        # zero on entry to a window's draw, cleared again by lds_engine_end_window
        self.deg = torch.zeros((count, S, int(nat.lib.lds_sample_ws_ints(n))), dtype=torch.int32, device=dev)
        self.row_ptr = torch.empty((count, S, n + 1), dtype=torch.int32, device=dev)
        self.col = torch.empty((count, S, max(cap, 1)), dtype=torch.int32, device=dev)
        self.s = torch.empty((count, S, n), dtype=torch.float32, device=dev)
        self.ell = torch.empty((count, S, n * 2 * ELL), dtype=torch.int32, device=dev)
        self.bptr = torch.empty((count, S, bptr_len), dtype=torch.int32, device=dev) if bptr_len else None
        self.graphs = [_Graph(n, cap, dev, views=(self.row_ptr[g], self.col[g], self.s[g], self.ell[g],
                                                  self.bptr[g] if bptr_len else None, self.bits[g]))
                       for g in range(count)]


class _Slot:
    """Tape of one inner step (or the outer step): graph + activations, the
    relu/dropout mask of layer 1 and (training with dropout) the dropped X
    values in CSR and CSC order."""

    def __init__(self, n: int, cap: int, dev, graph: "_Graph" = None, x_nnz: int = 0, samples: int = 1,
                 bptr_len: int = 0, words: int = 0):
        S = samples
        self.g = graph if graph is not None else _Graph(n, cap, dev, samples=S, bptr_len=bptr_len, words=words)
        for a in _ACT + ("dmask",):
            setattr(self, a, torch.zeros((S, n, HID), dtype=torch.float32, device=dev))
        self.xd_csr = torch.zeros((S, x_nnz), dtype=torch.float32, device=dev) if x_nnz else None
        self.xd_csc = torch.zeros((S, x_nnz), dtype=torch.float32, device=dev) if x_nnz else None
        self.lossrow = torch.zeros((S, n), dtype=torch.float32, device=dev)
        self.corrrow = torch.zeros((S, n), dtype=torch.float32, device=dev)


_POP8 = None


def _popcount(words: torch.Tensor) -> int:
    """Set bits in a device bit-row tensor (host sync; reporting only), by a
    byte table in 64 MB slices."""
    global _POP8
    if _POP8 is None or _POP8.device != words.device:
        _POP8 = torch.tensor([bin(i).count("1") for i in range(256)], dtype=torch.int32, device=words.device)
    b = words.reshape(-1).view(torch.uint8)
    tot = 0
    for i in range(0, b.numel(), 1 << 26):
        tot += int(_POP8[b[i:i + (1 << 26)].long()].sum().item())
    return tot


def _csr_of(dense: torch.Tensor):
    sp = dense.to_sparse_csr()
    return (sp.crow_indices().to(torch.int32).contiguous(), sp.col_indices().to(torch.int32).contiguous(),
            sp.values().to(torch.float32).contiguous())


def capture_into(graph, stream, body, pool=None, error_mode: str = "global", joins=()):
    """Capture body() into `graph` on `stream` (torch.cuda.CUDAGraph
    capture_begin / capture_end).

    An exception inside body() propagates ALONE, with the stream out of capture
    mode: every stream of `joins` that the capture forked (the engine's side
    stream) is joined back into `stream`, the capture is ended (an error of
    that end is dropped, it only restates the first one: unjoined work, an
    invalidated capture), the partial graph is reset, and then the first
    error is re-raised.  Without this, torch.cuda.graph's __exit__ raised
    hipErrorStreamCaptureUnjoined on top of the real cause (round-5 VERDICT,
    "What's weak" #8) and left the stream capturing."""
    with torch.cuda.stream(stream):
        if pool is None:
            graph.capture_begin(capture_error_mode=error_mode)
        else:
            graph.capture_begin(pool=pool, capture_error_mode=error_mode)
        try:
            body()
        except BaseException:
            _abort_capture(graph, stream, joins)
            raise
        graph.capture_end()


def _abort_capture(graph, stream, joins) -> None:
    for j in joins:
        try:
            with torch.cuda.stream(j):
                forked = torch.cuda.is_current_stream_capturing()
            if forked:
                stream.wait_stream(j)
        except Exception:  # noqa: BLE001  (cleanup only: the body's error is the one reported)
            pass
    try:
        graph.capture_end()
    except Exception:  # noqa: BLE001
        pass
    try:
        graph.reset()
    except Exception:  # noqa: BLE001
        pass


# outcome of one rank's window capture, agreed over ranks as the MIN
_CAPTURE_OK, _CAPTURE_RETRY_SPLIT, _CAPTURE_FATAL = 2, 1, 0


def _capture_status(err: Optional[BaseException]) -> int:
    """OK without an error; FATAL for an error of the engine's own launches
    or arguments (the same window fails in any capture form); else
    RETRY_SPLIT (a capture-specific failure, e.g. a collective library that
    cannot be captured: the split graphs keep the collective eager)."""
    if err is None:
        return _CAPTURE_OK
    if isinstance(err, (nat.NativeError, nat.DeviceError, ValueError, NotImplementedError, AssertionError,
                        KeyError, TypeError)):
        return _CAPTURE_FATAL
    return _CAPTURE_RETRY_SPLIT


def _collective_reducer(grad_reducer) -> bool:
    """The reducer is a collective over the default process group (the
    replicas' all-reduce: it carries the `capturable` attribute) and that
    group has more than one rank: every rank then captures its window in the
    same call, so the ranks can — and must — agree on the capture outcome."""
    if grad_reducer is None or getattr(grad_reducer, "capturable", None) is None:
        return False
    import torch.distributed as dist
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def _ranks_agree(status: int, device) -> int:
    """MIN of every rank's capture status, by an EAGER all-reduce (no graph
    holding a collective has been replayed yet, so no rank can be waiting
    inside one)."""
    import torch.distributed as dist
    on_dev = dist.get_backend() == "nccl"
    t = torch.tensor([status], dtype=torch.int32, device=device if on_dev else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return int(t.item())


class LdsEngine:
    """One replica of the LDS bilevel problem, resident on one GPU."""

    def __init__(self, x: torch.Tensor, y: torch.Tensor, train_mask: torch.Tensor, opt_mask: torch.Tensor,
                 theta: torch.Tensor, num_classes: int, dropout: float = 0.5, gcn_lr: float = 0.01,
                 gcn_wd: float = 5e-4, betas=(0.9, 0.999), eps: float = 1e-8, outer_lr: float = 1.0,
                 lr_decay: Optional[float] = None, tau: int = 5, generator: Optional[Generator] = None,
                 params: Optional["OrderedDict[str, torch.Tensor]"] = None, samples: int = 1,
                 long_rows: Optional[bool] = None, long_rows_kernel: str = "bitmask",
                 xt_splits: Optional[int] = None):
        nat.require_device(x, "LdsEngine")
        dev = x.device
        self.dev = dev
        self.S = int(samples)
        if not (1 <= self.S <= 4096):
            raise ValueError("samples must be in 1..4096")
        self.n, self.fin = int(x.shape[0]), int(x.shape[1])
        self.c = int(num_classes)
        if not (0 < self.c <= HID):
            raise NotImplementedError(f"LdsEngine supports 1..{HID} classes")
        n, fin, c = self.n, self.fin, self.c
        if theta.numel() != n * (n + 1) // 2 or theta.dtype != torch.float32 or not theta.is_contiguous():
            raise ValueError("theta must be the contiguous float32 packed upper triangle of an n×n matrix")
        self.theta = theta  # updated in place (the BernoulliGraphModel.probs storage)
        self.dropout = float(dropout)
        self.keep = float(np.float32(1.0) - np.float32(self.dropout))
        self.scale = float(np.float32(1.0) / np.float32(self.keep)) if self.keep > 0 else 0.0
        self.train_flag = 1 if self.dropout > 0.0 else 0
        self.hyper_np = np.array([gcn_lr, betas[0], betas[1], eps, gcn_wd], dtype=np.float64)
        self.betas_dev = torch.tensor([betas[0], betas[1], gcn_lr], dtype=torch.float64, device=dev)
        # Adam table: {lr/bc1, sqrt(bc2)} for steps adam_step+1+k (refreshed on device)
        self.adam_tab = torch.zeros(2 * _TAB_MAX, dtype=torch.float32, device=dev)
        self.gen = generator or Generator(0, 0)
        rep = self.gen.replica  # sample b is replica rep + b (tags + b)
        if rep + self.S > 0xFFFFFF:
            raise ValueError("replica tags exceed 24 bits")
        self.seed = self.gen.seed
        self.tag_graph = tag_for(TAG_GRAPH, rep)
        self.tag_x = tag_for(TAG_DROP_X, rep)
        self.tag_h = tag_for(TAG_DROP_H, rep)

        # data
        self.xrp, self.xcol, self.xval = _csr_of(x.float())
        self.xcp, self.xrow, self.xtval = _csr_of(x.float().t().contiguous())
        # position of each CSR entry of X in the CSC arrays (X is fixed)
        nnz = int(self.xcol.numel())
        rows = torch.repeat_interleave(torch.arange(n, device=dev), (self.xrp[1:] - self.xrp[:-1]).long())
        order = torch.argsort(self.xcol.long() * n + rows)
        self.csr2csc = torch.empty(nnz, dtype=torch.int32, device=dev)
        self.csr2csc[order] = torch.arange(nnz, dtype=torch.int32, device=dev)
        # row heads of X (lds_engine_x_linear xhead / xinfo): {p0, nnz} and the first 64 {column, value}
        rp0 = self.xrp[:-1].long()
        rnz = (self.xrp[1:] - self.xrp[:-1]).long()
        self.xinfo = torch.stack([rp0, rnz], 1).to(torch.int32).contiguous()
        self.xhead = self._head_of(rp0, rnz, self.xcol, self.xval)
        self.x_nnz = nnz if self.train_flag else 0
        # dense X (config 5: 20 000 entries per column): the W0 products run as
        # partial ranges of ~512 entries per wave instead of one wave per column
        col_avg = nnz / max(1, fin)
        if xt_splits is None:
            xt_splits = 1 if col_avg < 2048 else min(64, int(np.ceil(col_avg / 512)))
        self.set_xt_splits(xt_splits)
        self.label = y.to(device=dev, dtype=torch.int32).contiguous()
        self.train_mask = train_mask.to(device=dev, dtype=torch.uint8).contiguous()
        self.opt_mask = opt_mask.to(device=dev, dtype=torch.uint8).contiguous()
        # node flags carried in every ELL entry (include/ldsgnn.h): bit 0 train, bit 1 opt
        self.nflag = (self.train_mask | (self.opt_mask << 1)).contiguous()
        self.inv_train = float(np.float32(1.0) / np.float32(int(train_mask.sum())))
        self.inv_opt = float(np.float32(1.0) / np.float32(int(opt_mask.sum())))

        # parameter layout
        self.np = fin * HID + HID + c * HID + c
        self.off_b0 = fin * HID
        self.off_w1 = self.off_b0 + HID
        self.off_b1 = self.off_w1 + c * HID
        self.n_wd = self.off_w1  # group 0 = layer_in (weight + bias)

        # device scalars {u32 graph_ctr, u32 fwd_ctr, i32 adam_step, i32 hyper, f64 lr, f64 decay,
        # u32 error, u32 pad}: `error` is the device error word the window fills report into
        assert nat.lib.lds_engine_scalars_size() == 40
        self.scalars = torch.zeros(40, dtype=torch.uint8, device=dev)
        self._i32 = self.scalars[:16].view(torch.int32)
        self._f64 = self.scalars[16:32].view(torch.float64)
        self._err = self.scalars[32:36].view(torch.int32)
        self._i32.copy_(torch.tensor([self.gen.graph_counter, self.gen.forward_counter, 0, 0], dtype=torch.int32))
        self._f64.copy_(torch.tensor([outer_lr, 1.0 if lr_decay is None else lr_decay], dtype=torch.float64))

        # long rows (dense θ, BASELINE config 5): the aggregations run as a
        # pre-pass whose Â·Z the fused kernels read instead of aggregating
        # in-kernel — the bitmask aggregation on the int8 matrix cores
        # (lds_aggregate_bitmask, no CSR is built), the CSR spill-pass SpMM
        # (lds_spmm_norm_dense, long_rows_kernel="csr") or the column-blocked
        # LDS SpMM over CSR (lds_spmm_norm_blocked, long_rows_kernel="blocked").
        # Decided once from θ's expected degree 1 + 2·Σ_{i<j} clamp(θ_ij) / n.
        if long_rows is None:
            tsum = float(theta.clamp(0, 1).double().sum().item())
            diag = float(theta.view(-1)[torch.arange(n, device=dev) * (2 * n + 1 - torch.arange(n, device=dev)) // 2]
                         .clamp(0, 1).double().sum().item())
            long_rows = n >= 1024 and 1.0 + 2.0 * (tsum - diag) / n >= 256.0
        self.long_rows = bool(long_rows)
        # two-hop loss kernels (lds_engine_fwd2_bwd2 / lds_engine_rev_bc): need the
        # ELL head with node flags, i.e. in-kernel aggregation (short rows)
        self.two_hop = not self.long_rows
        # the outer step's loss (opt mask, ~2x the train rows) as one two-hop
        # launch too.  Round 2 measured the separate launches faster (more
        # masked neighbours per row -> more rounds); with the two-hop kernels'
        # own row plan (rows with many masked neighbours on blocks of their own)
        # the one launch now wins by ≈2 µs per window at Cora (round 5: 14.52k
        # against 14.48k steps/s, 56 launches per window; bench --two-hop-outer)
        self.two_hop_outer = True
        # the exchange path's SGD + next-window draw (lds_sgd_sample_graphs)
        # with the replica samples split over more blocks (per-tile counters;
        # same θ and draws): False = one block per tile, the round-4 form
        self.sgd_draw_split = True
        # its per-tile counters (zero, and every call leaves them zero), allocated
        # here rather than on first use, which may fall inside a graph capture
        self._sgd_tiles = torch.zeros(int(nat.lib.lds_sgd_tile_ints(n)), dtype=torch.int32, device=theta.device)
        self._sgd_tiles_checked = False
        if self.long_rows and self.S > 1:
            raise NotImplementedError("long-row (dense θ) mode runs one replica sample per engine")
        if long_rows_kernel not in ("bitmask", "csr", "blocked"):
            raise ValueError("long_rows_kernel: 'bitmask', 'csr' or 'blocked'")
        self.bitmask_agg = self.long_rows and long_rows_kernel == "bitmask"
        self.dense_agg = self.long_rows and long_rows_kernel == "csr"
        if self.dense_agg and n > nat.lib.lds_spmm_dense_max_n():
            raise NotImplementedError(f"long_rows_kernel='csr': n <= {nat.lib.lds_spmm_dense_max_n()}")
        self.agg_splits = 0  # bitmask aggregation: its partial arrays, summed by the consumers
        # graph buffers: CSR column capacity n² per graph (int32 positions);
        # none when the bitmask aggregation reads the sampled bits directly
        # (the per-graph column stride rounded up to 4 ints: every graph's col
        # then starts 16-byte aligned, as lds_spmm_norm_dense requires, also
        # for odd n)
        cap = (n * n + 3) & ~3
        if not self.bitmask_agg and cap >= (1 << 31):
            raise NotImplementedError("LdsEngine needs n² < 2^31 (int32 CSR positions)")
        self.cap = 0 if self.bitmask_agg else cap
        self.bptr_len = n * (nat.lib.lds_spmm_block_count(n) + 1) \
            if self.long_rows and not (self.bitmask_agg or self.dense_agg) else 0
        self.words = nat.lib.lds_bitmask_words(n)
        S = self.S
        self.deg = torch.empty((S, int(nat.lib.lds_sample_ws_ints(n))), dtype=torch.int32, device=dev)
        self._ws_clean = True  # gbatch.deg is zero (fresh, or cleared by the last end_window)
        # prefetched draws (capture_window(prefetch=True)): the hyper step's
        # θ-grad kernel also draws the NEXT window's graphs from the θ it writes
        # (lds_theta_grad_sgd_draw, degrees into deg_next, moved to gbatch.deg
        # by end_window), and the next window only fills CSR / s / ELL
        self.prefetch_draw = False
        self._prefetched = False
        self._deg_next = None

        # tape
        self.tau = max(1, int(tau))
        self.cw = (c + 3) & ~3
        self.kg = 2 * HID + 2 * self.cw  # factor columns per inner graph
        self.slots: List[_Slot] = []
        self.w: List[torch.Tensor] = []
        self.m: List[torch.Tensor] = []
        self.v: List[torch.Tensor] = []
        self.gp: List[torch.Tensor] = []
        self.gbatch = _GraphBatch(self.tau + 1, n, self.words, self.cap, dev, samples=S, bptr_len=self.bptr_len)
        if self.long_rows:
            self.agg = torch.zeros((S, n, HID), dtype=torch.float32, device=dev)
            if self.bitmask_agg:
                self.agg_ws = torch.empty(int(nat.lib.lds_bitmask_agg_ws_bytes(n)), dtype=torch.uint8, device=dev)
                self.agg_part_off = int(nat.lib.lds_bitmask_agg_part_offset(n))
                self.agg_splits = int(nat.lib.lds_bitmask_agg_splits(n))
            elif self.dense_agg:
                self.agg_ws = torch.empty(int(nat.lib.lds_spmm_dense_ws_bytes(n)), dtype=torch.uint8, device=dev)
            else:
                nb = nat.lib.lds_spmm_block_count(n)
                self.spmm_part = torch.zeros((nb, n, HID), dtype=torch.float32, device=dev)
        # per-step HIP graphs (inner_step_graphed / hyper_step_graphed): keyed
        # captures, keys seen once, and the buffer-layout version they hold
        self._step_graphs, self._step_seen, self._layout_version = {}, set(), 0
        self._grow(self.tau)
        self.outer = _Slot(n, self.cap, dev, graph=self.gbatch.graphs[self.tau], x_nnz=self.x_nnz, samples=S)
        self.t = 0  # inner steps in the current window
        self.pending_graph = 0
        self.pending_fwd = 0

        # reverse-pass buffers
        z = lambda: torch.zeros((S, n, HID), dtype=torch.float32, device=dev)  # noqa: E731
        self.dh0bar, self.dh1dbar, self.dh2bar, self.h1dbar = z(), z(), z(), z()
        self.obar, self.h2bar, self.y0bar, self.h0bar = z(), z(), z(), z()
        zp = lambda: torch.zeros((S, self.np), dtype=torch.float32, device=dev)  # noqa: E731
        self.wbar, self.mbar, self.vbar, self.gbar, self.g = zp(), zp(), zp(), zp(), zp()
        self._row_plan()
        # first-stage partials of the fused reductions: 16 rows per block, plus
        # one block per heavy row of the plan
        self.nred = (n + 15) // 16 + self.n_heavy
        self.partials = torch.zeros((S, self.nred, _RED_LEN), dtype=torch.float32, device=dev)
        self._alloc_factors()
        self.grad = torch.zeros_like(theta)
        self.keep_grad = True  # write dθ (θ.grad) even when it is fused with the update
        # outer_update(grad): replaces the SGD + clamp step on θ — a graph model
        # whose θ is a function of its own parameters (the embedding model)
        # takes dθ, steps its optimizer and rewrites self.theta in place
        self.outer_update = None
        # theta_fn(counter) -> θ of one draw (set_theta_fn): θ redrawn per
        # sample, as a GAE proposal with dropout makes it (None: one θ)
        self.theta_fn = None
        self._fwd_of = {}  # inner step t -> the forward counter offset its classifier forward took
        # grad_reducer(grad): the default exchange of a hyper step (e.g. the
        # all-reduce mean of dθ over ranks, ldsgnn.replicas); when set, dθ is
        # written, reduced, then SGD + clamp runs (the assembly is not fused
        # with the update), and captures split at it
        self.grad_reducer = None
        # band-sharded replicas (set_band_shards): the long-row engine's
        # exchange at N > 1 as factor all-gather + band update + band draws
        self.shards = None
        self._allbits = None
        # dθ assembly split per graph: chunks of finished graphs run on a side
        # stream beside the (latency-bound) reverse pass.  Off by default: on
        # MI355X the replayed graph did not overlap the branches and the
        # chunks' read-modify-write of dθ cost 2.3x the single launch (r01).
        self.split_theta_grad = False
        # window draw split (replica samples): graph 0 on the main stream, the
        # window's other graphs on the side stream beside inner step 0 (a
        # captured graph keeps the fork / join as edges)
        self.async_draw = False
        self._draw_pending = False
        # prefetched window fill launched together with the first X product
        # (lds_engine_fill_x_linear); the fill is deferred until that launch
        self.fuse_fill = True
        self._pending_fill = None
        # factor planes for the direct-staged θ-grad (form "bf16x3-direct", and
        # the by-shape default on Cora-sized grids): see _planes_window
        self.uv_planes = True
        self._planes_now = False
        # θ-grad assembly form of this engine's launches (ldsgnn.ops.THETA_GRAD_FORMS
        # name; None: the module default ops.theta_grad_form() at launch time)
        self.theta_form = None
        self.side = torch.cuda.Stream(dev)
        self.metrics = torch.zeros((self.tau + 1, S, 2), dtype=torch.float32, device=dev)
        self._graph_capture = None
        if params is not None:
            self.set_params(params)
        self.reset_optimizer()

    # ------------------------------------------------------------------ setup
    def _form_name(self) -> str:
        from .ops import theta_grad_form
        return self.theta_form if self.theta_form is not None else theta_grad_form()

    def _form(self) -> int:
        """The C-ABI `form` argument of this engine's θ-grad launches."""
        from .ops import form_code
        return form_code(self._form_name())

    def _alloc_factors(self):
        """U, V: n × (S·ldk), sample b in columns [b·ldk, (b+1)·ldk); R: [S, n]."""
        self._layout_version += 1  # captured step graphs are stale
        self.ktot = self.tau * self.kg + HID + self.cw
        self.ldk = (self.ktot + 3) & ~3
        self.ldu = self.S * self.ldk  # row stride of U / V (the kernels' `ldk` argument)
        self.U = torch.zeros((self.n, self.ldu), dtype=torch.float32, device=self.dev)
        self.V = torch.zeros_like(self.U)
        self.R = torch.zeros((self.S, self.n), dtype=torch.float32, device=self.dev)
        # the same factors as split-bf16 planes in the direct-staged θ-grad's
        # 128-row-tile layout (include/ldsgnn.h lds_split_planes_t128), written
        # by the factor producers instead of U / V in windows that assemble dθ
        # with lds_theta_grad_direct (_planes_window); allocated on first use
        self.Up = self.Vp = None
        self._make_batches()

    # rows expected to have more than this many entries get a block of their own
    HEAVY_DEGREE = 64
    # ... and so do rows expected to have more than this many neighbours in a
    # loss mask (the two-hop kernels recompute each such neighbour's row)
    HEAVY_MASKED = 4

    def _row_plan(self):
        """The aggregating kernels' row plan (include/ldsgnn.h LdsBatch): rows
        whose expected degree 1 + Σ_j clamp(θ_ij, 0, 1) exceeds HEAVY_DEGREE
        (and 4 × the median degree),
        or whose expected count of train (or opt) neighbours, self included,
        exceeds HEAVY_MASKED, run on a block of their own.  Decided once from θ
        at construction: it changes speed only (a row of any degree is
        aggregated correctly either way).  Long-row mode (pre-aggregated Â·Z)
        has no plan."""
        n = self.n
        self.heavy_flag = torch.zeros(n, dtype=torch.uint8, device=self.dev)
        self.heavy_flag2 = torch.zeros(n, dtype=torch.uint8, device=self.dev)
        if self.long_rows:
            self.heavy_rows = self.heavy_rows2 = torch.zeros(1, dtype=torch.int32, device=self.dev)
            self.n_heavy = self.n_heavy2 = 0
            return
        i = torch.arange(n, device=self.dev)
        deg = torch.ones(n, device=self.dev)
        mt = self.train_mask.float()
        et = mt.clone()  # expected train neighbours (self-loop included)
        step = max(1, (1 << 24) // n)  # rows per chunk of the packed triangle
        for r0 in range(0, n, step):
            r1 = min(n, r0 + step)
            lo, hi = r0 * (2 * n - r0 + 1) // 2, r1 * (2 * n - r1 + 1) // 2
            rows = torch.repeat_interleave(i[r0:r1], n - i[r0:r1])  # row of each packed entry
            cols = rows + (torch.arange(lo, hi, device=self.dev) - (rows * (2 * n - rows + 1)) // 2)
            p = self.theta[lo:hi].clamp(0.0, 1.0) * (rows != cols)
            deg.index_add_(0, rows, p).index_add_(0, cols, p)
            et.index_add_(0, rows, p * mt[cols]).index_add_(0, cols, p * mt[rows])
        # a block per row pays off for the few hubs of a skewed graph; when
        # the typical row is long (config 5's sparse variant: every row ~100)
        # a wave per row walks it and the per-row blocks would only multiply
        # the fused reductions' partials (20 000 → 1 final block summing 21 k)
        thr = max(float(self.HEAVY_DEGREE), 4.0 * float(deg.median()))
        heavy = deg > thr
        # the two-hop kernels' own plan (their LdsBatch, bt2): also rows with
        # many train neighbours (no block reductions there, so nred is unaffected)
        heavy2 = heavy | (et > self.HEAVY_MASKED)
        self.heavy_rows2 = i[heavy2].to(torch.int32).contiguous() if bool(heavy2.any()) else \
            torch.zeros(1, dtype=torch.int32, device=self.dev)
        self.heavy_flag2[heavy2] = 1
        self.n_heavy2 = int(heavy2.sum())
        self.heavy_rows = i[heavy].to(torch.int32).contiguous() if bool(heavy.any()) else \
            torch.zeros(1, dtype=torch.int32, device=self.dev)
        self.heavy_flag[heavy] = 1
        self.n_heavy = int(heavy.sum())

    def _make_batches(self):
        """LdsBatch strides for this engine's layout (kept alive on self)."""
        n, S = self.n, self.S

        def mk(xval_stride):
            return nat.LdsBatch(samples=S, tag_step=1, act=n * HID, row=n, rp=n + 1, col=self.cap,
                                ell=n * 2 * ELL, par=self.np, xval=xval_stride, xd=self.x_nnz, uv=self.ldk,
                                part=self.nred * _RED_LEN, met=2, heavy_rows=nat.ptr(self.heavy_rows),
                                heavy_flag=nat.ptr(self.heavy_flag), n_heavy=self.n_heavy,
                                agg_splits=self.agg_splits)
        self._bt = mk(0)  # X values argument = the shared X
        self._btx = mk(self.x_nnz if self.train_flag else 0)  # X values argument = the slot's stored Xd
        self._bt2 = mk(0)  # the two-hop kernels: their own row plan
        self._bt2.heavy_rows, self._bt2.heavy_flag = nat.ptr(self.heavy_rows2), nat.ptr(self.heavy_flag2)
        self._bt2.n_heavy = self.n_heavy2
        self.bt = nat.batch_ptr(self._bt)
        self.btx = nat.batch_ptr(self._btx)
        self.bt2 = nat.batch_ptr(self._bt2)

    def _grow(self, slots: int):
        self._layout_version += 1
        if slots > _TAB_MAX:
            raise NotImplementedError(f"LdsEngine: at most {_TAB_MAX} inner steps per hyper step")
        while len(self.slots) < slots:
            t = len(self.slots)
            g = self.gbatch.graphs[t] if t < self.gbatch.count - 1 else None
            self.slots.append(_Slot(self.n, self.cap, self.dev, graph=g, x_nnz=self.x_nnz, samples=self.S,
                                    bptr_len=self.bptr_len, words=self.words))
        while len(self.w) < slots + 1:
            for lst in (self.w, self.m, self.v):
                lst.append(torch.zeros((self.S, self.np), dtype=torch.float32, device=self.dev))
        while len(self.gp) < slots:
            self.gp.append(torch.zeros((self.S, self.np), dtype=torch.float32, device=self.dev))

    def _stream(self) -> int:
        return nat.stream_of(self.dev)

    def _views(self, flat: torch.Tensor):
        """(W0ᵀ, b0, W1, b1) slices of a flat [.., np] parameter vector; their
        data pointers address sample 0 (kernels add b·np)."""
        c = self.c
        return (flat[..., : self.off_b0], flat[..., self.off_b0:self.off_w1], flat[..., self.off_w1:self.off_b1],
                flat[..., self.off_b1:self.off_b1 + c])

    def _write_params(self, flat: torch.Tensor, params) -> None:
        w0t, b0, w1, b1 = self._views(flat)
        with torch.no_grad():
            w0t.view(self.fin, HID).copy_(params["layer_in.fc.weight"].detach().t())
            b0.copy_(params["layer_in.fc.bias"].detach())
            w1.view(self.c, HID).copy_(params["layer_out.fc.weight"].detach())
            b1.copy_(params["layer_out.fc.bias"].detach())

    def set_params(self, params):
        """Load reference-layout params (layer_in.fc.weight [16, fin], ...)
        into every replica sample (all chains start from the same GCN)."""
        self._drop_prefetch()
        for b in range(self.S):
            self._write_params(self.w[0][b], params)
        self.t = 0

    def flat_params(self, sample: int = 0) -> torch.Tensor:
        """A copy of the current flat parameter vector of one sample."""
        return self.w[self.t][sample].clone()

    def params_from_flat(self, flat: torch.Tensor) -> "OrderedDict[str, torch.Tensor]":
        w0t, b0, w1, b1 = self._views(flat)
        return OrderedDict([
            ("layer_in.fc.weight", w0t.reshape(self.fin, HID).t().contiguous()),
            ("layer_in.fc.bias", b0.clone()),
            ("layer_out.fc.weight", w1.reshape(self.c, HID).clone()),
            ("layer_out.fc.bias", b1.clone()),
        ])

    def empirical_mean(self, flat: torch.Tensor, n_samples: int, val_mask: torch.Tensor,
                       test_mask: torch.Tensor):
        """empirical_mean_loss (src/utils/evaluation.py:51-84) with the fused
        kernels: n_samples graphs drawn from θ (they take graph counters, as
        the reference's samples take RNG draws), eval-mode forward with the
        flat parameters, NLL / accuracy on the validation and test masks,
        averaged over samples; one host sync.  Single-sample engines."""
        self._flush_fill()
        self._drop_prefetch()
        if self.S != 1:
            raise NotImplementedError("empirical_mean runs on single-sample engines")
        if self.shards is not None and self.shards.world > 1 and not self._theta_whole:
            raise RuntimeError("empirical_mean: band-sharded θ is current only in this rank's band; "
                               "call sync_theta() first")
        if not self.long_rows:
            return self._empirical_mean_batched(flat, n_samples, val_mask, test_mask)
        return self._empirical_mean_seq(flat, n_samples, val_mask, test_mask)

    def _empirical_mean_seq(self, flat: torch.Tensor, n_samples: int, val_mask: torch.Tensor,
                            test_mask: torch.Tensor):
        """empirical_mean one evaluation graph at a time (long rows: the
        aggregation pre-pass buffers are single-sample)."""
        st, n, c = self._stream(), self.n, self.c
        if getattr(self, "_eval", None) is None:
            self._eval = _Slot(n, self.cap, self.dev, x_nnz=0, samples=1, bptr_len=self.bptr_len, words=self.words)
            self._eval_w = torch.zeros((1, self.np), dtype=torch.float32, device=self.dev)
            self._eval_rows = torch.zeros((2, n), dtype=torch.float32, device=self.dev)
        sl, g = self._eval, self._eval.g
        self._eval_w[0].copy_(flat)
        vm = val_mask.to(device=self.dev, dtype=torch.uint8).contiguous()
        tm = test_mask.to(device=self.dev, dtype=torch.uint8).contiguous()
        inv_v = float(np.float32(1.0) / np.float32(int(val_mask.sum())))
        inv_t = float(np.float32(1.0) / np.float32(int(test_mask.sum())))
        sums = []
        for _ in range(n_samples):
            self._sample(g)
            self._forward(sl, self._eval_w, vm, inv_v, 0, 0)  # val rows -> sl.lossrow / corrrow
            nat.call("lds_engine_fwd_layer2", nat.ptr(g.row_ptr), nat.ptr(g.col), nat.ptr(g.s), nat.ptr(g.ell), n,
                     nat.ptr(sl.h2), 0, 0, 0, nat.ptr(self.label), nat.ptr(tm), inv_t, nat.ptr(self._eval_rows[0]),
                     nat.ptr(self._eval_rows[1]), c, self._agg(g, sl.h2), self.bt, st)
            sums.append(torch.stack([sl.lossrow[0].sum(), sl.corrrow[0].sum(), self._eval_rows[0].sum(),
                                     self._eval_rows[1].sum()]))
        host = torch.stack(sums).double().cpu().numpy()
        self.check_device_error()
        return (float(np.mean(host[:, 0] * inv_v)), float(np.mean(host[:, 1] * inv_v)),
                float(np.mean(host[:, 2] * inv_t)), float(np.mean(host[:, 3] * inv_t)))

    def _empirical_mean_batched(self, flat: torch.Tensor, n_samples: int, val_mask: torch.Tensor,
                                test_mask: torch.Tensor):
        """empirical_mean with the n_samples evaluation graphs as one batch
        (short rows): one lds_sample_graphs_multi launch set draws them with
        the counters the sequential draws would take (graph g: counter
        base + pending + g), and every eval-mode forward kernel runs once with
        grid.y = sample over LdsBatch strides whose parameter stride is 0 (all
        samples read the same weights)."""
        st, n, c, E = self._stream(), self.n, self.c, int(n_samples)
        if getattr(self, "_evb_E", 0) != E:
            self._evb = _Slot(n, self.cap, self.dev, x_nnz=0, samples=E, bptr_len=0, words=self.words)
            self._evb_deg = torch.empty((E, int(nat.lib.lds_sample_ws_ints(n))), dtype=torch.int32, device=self.dev)
            self._evb_rows = torch.zeros((2, E, n), dtype=torch.float32, device=self.dev)
            self._evb_w = torch.zeros((1, self.np), dtype=torch.float32, device=self.dev)
            self._evb_bt_obj = nat.LdsBatch(samples=E, tag_step=1, act=n * HID, row=n, rp=n + 1, col=self.cap,
                                            ell=n * 2 * ELL, par=0, xval=0, xd=0, uv=0, part=0, met=2)
            self._evb_bt = nat.batch_ptr(self._evb_bt_obj)
            self._evb_E = E
        sl, g, bt = self._evb, self._evb.g, self._evb_bt
        self._evb_w[0].copy_(flat)
        vm = val_mask.to(device=self.dev, dtype=torch.uint8).contiguous()
        tm = test_mask.to(device=self.dev, dtype=torch.uint8).contiguous()
        inv_v = float(np.float32(1.0) / np.float32(int(val_mask.sum())))
        inv_t = float(np.float32(1.0) / np.float32(int(test_mask.sum())))
        nat.call("lds_sample_graphs_multi", nat.ptr(self.theta), n, self.seed, self.tag_graph, 1,
                 nat.ptr(self.scalars), self.pending_graph, E, 1, nat.ptr(g.bits), self.words,
                 nat.ptr(self._evb_deg), nat.ptr(g.row_ptr), nat.ptr(g.col), self.cap, nat.ptr(g.s),
                 nat.ptr(g.ell), nat.ptr(self.nflag), 0, self._err_ptr(), st)
        self.pending_graph += E
        self._forward(sl, self._evb_w, vm, inv_v, 0, 0, bt=bt)  # val rows -> sl.lossrow / corrrow [E, n]
        rl, rc = self._evb_rows[0], self._evb_rows[1]
        nat.call("lds_engine_fwd_layer2", nat.ptr(g.row_ptr), nat.ptr(g.col), nat.ptr(g.s), nat.ptr(g.ell), n,
                 nat.ptr(sl.h2), 0, 0, 0, nat.ptr(self.label), nat.ptr(tm), inv_t, nat.ptr(rl), nat.ptr(rc), c, 0,
                 bt, st)
        host = torch.stack([sl.lossrow.sum(1), sl.corrrow.sum(1), rl.sum(1), rc.sum(1)], 1).double().cpu().numpy()
        self.check_device_error()
        return (float(np.mean(host[:, 0] * inv_v)), float(np.mean(host[:, 1] * inv_v)),
                float(np.mean(host[:, 2] * inv_t)), float(np.mean(host[:, 3] * inv_t)))

    def get_params(self, sample: int = 0) -> "OrderedDict[str, torch.Tensor]":
        w0t, b0, w1, b1 = self._views(self.w[self.t][sample])
        return OrderedDict([
            ("layer_in.fc.weight", w0t.view(self.fin, HID).t().contiguous()),
            ("layer_in.fc.bias", b0.clone()),
            ("layer_out.fc.weight", w1.view(self.c, HID).clone()),
            ("layer_out.fc.bias", b1.clone()),
        ])

    def reset_optimizer(self):
        """InnerProblemTrainer.reset_optimizer: fresh Adam state, step 0."""
        self._flush()
        cur = self.t
        if cur != 0:
            self.w[0].copy_(self.w[cur])
        self.m[0].zero_()
        self.v[0].zero_()
        self._i32[2:3].zero_()
        self._refresh_adam_table()
        self.t = 0

    def _tab_count(self) -> int:
        return max(1, len(self.slots))

    def _refresh_adam_table(self):
        nat.call("lds_engine_adam_table", nat.ptr(self.scalars), nat.ptr(self.betas_dev), nat.ptr(self.adam_tab),
                 self._tab_count(), self._stream())

    def _flush(self, hypers: int = 0):
        """Apply pending counter offsets to the device scalars."""
        if self.pending_graph or self.pending_fwd or self.t or hypers:
            nat.call("lds_engine_advance", nat.ptr(self.scalars), self.pending_graph, self.pending_fwd, self.t,
                     hypers, self._stream())
            if self.t:
                self._refresh_adam_table()
        self.pending_graph = 0
        self.pending_fwd = 0

    def sync_generator(self):
        """Write the device draw counters back to the host Generator (sync)."""
        self._flush_counters_only()
        vals = self._i32.cpu().tolist()
        self.gen.graph_counter, self.gen.forward_counter = int(vals[0]), int(vals[1])

    def _flush_counters_only(self):
        if self.pending_graph or self.pending_fwd:
            nat.call("lds_engine_advance", nat.ptr(self.scalars), self.pending_graph, self.pending_fwd, 0, 0,
                     self._stream())
        self.pending_graph = 0
        self.pending_fwd = 0

    # --------------------------------------------------------------- pieces
    def _sample(self, g: _Graph, theta: torch.Tensor = None):
        """Draw the next graph of every replica sample into `g` (from `theta`,
        default self.theta)."""
        self._drop_prefetch()
        if self.shards is not None and theta is None:
            self._sharded_draw(g.bits, self.deg, g.s, (g.row_ptr, g.col, g.ell), 1, self.pending_graph)
            self._block_ptrs([g])
            self.pending_graph += 1
            return
        nat.call("lds_sample_graphs_multi", nat.ptr(self.theta if theta is None else theta), self.n, self.seed, self.tag_graph, 1,
                 nat.ptr(self.scalars), self.pending_graph, 1, self.S, nat.ptr(g.bits), self.words,
                 nat.ptr(self.deg), nat.ptr(g.row_ptr), self._col_arg(g.col), self.cap, nat.ptr(g.s),
                 nat.ptr(g.ell), nat.ptr(self.nflag), 0, self._err_ptr(), self._stream())
        self._block_ptrs([g])
        self.pending_graph += 1

    def _col_arg(self, col: torch.Tensor) -> int:
        return 0 if self.bitmask_agg else nat.ptr(col)  # NULL: no CSR (bitmask aggregation)

    def _block_ptrs(self, graphs):
        if self.bptr_len:
            for g in graphs:
                nat.call("lds_csr_block_ptr", nat.ptr(g.row_ptr), nat.ptr(g.col), self.n, nat.ptr(g.bptr),
                         self._stream())

    def _agg(self, g: _Graph, z: torch.Tensor) -> int:
        """Long rows: Â·Z into self.agg by the bitmask aggregation, the CSR
        spill-pass SpMM or the column-blocked SpMM (the fused kernel then reads
        it); short rows: 0 (aggregate in-kernel)."""
        if not self.long_rows:
            return 0
        if self.bitmask_agg:  # the split partials; the consuming kernel sums them (LdsBatch.agg_splits)
            nat.call("lds_aggregate_bitmask_partials", nat.ptr(g.bits), self.words, nat.ptr(g.s), self.n,
                     nat.ptr(z), HID, nat.ptr(self.agg_ws), self._stream())
            return nat.ptr(self.agg_ws) + self.agg_part_off
        if self.dense_agg:
            nat.call("lds_spmm_norm_dense", nat.ptr(g.row_ptr), nat.ptr(g.col), nat.ptr(g.s), self.n, nat.ptr(z),
                     HID, nat.ptr(self.agg), HID, 0, nat.ptr(self.agg_ws), 0, 1, 0, self._stream())  # (the
            # engine's own fill: canonical columns, the unchecked form)
            return nat.ptr(self.agg)
        nat.call("lds_spmm_norm_blocked", nat.ptr(g.bptr), nat.ptr(g.col), nat.ptr(g.s), self.n, nat.ptr(z), HID,
                 nat.ptr(self.agg), HID, 0, nat.ptr(self.spmm_part), self._stream())
        return nat.ptr(self.agg)

    def _forward(self, sl: _Slot, w: torch.Tensor, mask, inv_count, train: int, fwd_off: int, bt=None,
                 loss_in_backward: bool = False, bt_l1=None):
        """X-linear, layer 1 and (unless loss_in_backward: the two-hop
        backward computes it) the loss layer."""
        st, n, c = self._stream(), self.n, self.c
        bt = self.bt if bt is None else bt
        w0t, b0, w1, b1 = self._views(w)
        g = sl.g
        # training forwards keep Xd (CSR + CSC order) and the relu/dropout mask
        # on the tape: the step's later products read them instead of redrawing
        keep_xd = train and sl.xd_csr is not None
        xd = (nat.ptr(sl.xd_csr), nat.ptr(sl.xd_csc), nat.ptr(self.csr2csc)) if keep_xd else (0, 0, 0)
        xargs = (nat.ptr(self.xrp), nat.ptr(self.xcol), nat.ptr(self.xval), n, nat.ptr(w0t), nat.ptr(b0),
                 nat.ptr(sl.h0), self.seed, self.tag_x, nat.ptr(self.scalars), fwd_off, train, self.keep,
                 self.scale, *xd, nat.ptr(self.xhead), nat.ptr(self.xinfo), 1, bt, st)
        if self._pending_fill is not None and bt == self.bt:  # the window's fill rides in this launch
            nat.call("lds_engine_fill_x_linear", *self._pending_fill, *xargs)
            self._pending_fill = None
        else:
            self._flush_fill()
            nat.call("lds_engine_x_linear", *xargs)
        nat.call("lds_engine_fwd_layer1", nat.ptr(g.row_ptr), nat.ptr(g.col), nat.ptr(g.s), nat.ptr(g.ell), n, nat.ptr(sl.h0),
                 nat.ptr(sl.y0), nat.ptr(sl.h1d), nat.ptr(sl.h2), nat.ptr(w1), nat.ptr(b1), c, self.seed,
                 self.tag_h, nat.ptr(self.scalars), fwd_off, train, self.keep, self.scale, nat.ptr(sl.dmask),
                 self._agg(g, sl.h0), bt if bt_l1 is None else bt_l1, st)
        if loss_in_backward and self.two_hop:
            return
        nat.call("lds_engine_fwd_layer2", nat.ptr(g.row_ptr), nat.ptr(g.col), nat.ptr(g.s), nat.ptr(g.ell), n, nat.ptr(sl.h2),
                 nat.ptr(sl.o), nat.ptr(sl.p), nat.ptr(sl.d_o), nat.ptr(self.label), nat.ptr(mask), inv_count,
                 nat.ptr(sl.lossrow), nat.ptr(sl.corrrow), c, self._agg(g, sl.h2), bt, st)

    def set_xt_splits(self, splits: int):
        """Entry ranges per X column for the W0 products (1: one wave per
        column; chosen from X's density at construction).  Call between
        windows, before capture_window."""
        self.xt_splits = max(1, int(splits))
        self.xt_part = (torch.zeros((self.S, self.xt_splits, self.fin, HID), dtype=torch.float32, device=self.dev)
                        if self.xt_splits > 1 else None)
        self._xt_plan()
        self._layout_version = getattr(self, "_layout_version", 0) + 1  # captured step graphs are stale

    def set_xt_pair(self, mode: int):
        """W0 products (lds_engine_xt_adam) over pairs of replica samples, two
        per wave sharing one walk of X's column indices (same sums): 0 by
        shape (the library's rule), 1 off, 2 on (an even sample count; the
        column plan then has no heavy columns).  Call between windows, before
        capture_window."""
        if mode not in (0, 1, 2):
            raise ValueError("xt_pair: 0 (by shape), 1 (off) or 2 (on)")
        if mode == 2 and self.S % 2:
            raise ValueError("xt_pair = 2 needs an even number of samples")
        self.xt_pair = mode
        self._btx.xt_pair = mode
        self._xt_plan()
        self._layout_version += 1  # captured step graphs are stale

    def _xt_plan(self):
        """lds_engine_xt_adam's column plan (X is fixed): the columns with more
        than 128 entries first (a 1024-thread block each), then the rest (one
        wave each); with split products (xt_splits > 1) no heavy columns."""
        lens = (self.xcp[1:] - self.xcp[:-1]).long()
        # up to 8 batched samples the long columns still set the time (Cora,
        # per call: S = 4 9.9 vs 12.5 µs, S = 8 16.1 vs 16.6 with heavy
        # blocks); from 16 on every column stays one wave, where the
        # 1024-thread heavy blocks only fragment the CU (Cora S = 16 31.0 vs
        # 30.9; Citeseer S = 16 73.4 vs 59.6 µs)
        # (and none when the W0 products pair samples per wave: set_xt_pair(2))
        heavy = (lens > 128) if self.xt_splits <= 1 and self.S <= 8 and getattr(self, "xt_pair", 0) != 2 \
            else torch.zeros_like(lens, dtype=torch.bool)
        idx = torch.arange(self.fin, device=self.dev)
        if self.xt_splits <= 1:
            # the other columns by length: > 32 entries one wave each, 17-32
            # two per wave, <= 16 four per wave (same sums, fewer waves)
            one = ~heavy & (lens > 32)
            two = ~heavy & (lens > 16) & (lens <= 32)
            four = ~heavy & (lens <= 16)
        else:
            one, two, four = ~heavy, torch.zeros_like(heavy), torch.zeros_like(heavy)
        self.xt_order = torch.cat([idx[heavy], idx[one], idx[two], idx[four]]).to(torch.int32).contiguous()
        self.xt_heavy = int(heavy.sum())
        self.xt_n1, self.xt_n2 = int(one.sum()), int(two.sum())
        # column heads by plan slot (lds_engine_xt_adam xtinfo / xthead)
        f = self.xt_order.long()
        p0 = self.xcp[f].long()
        nz = (self.xcp[f + 1] - self.xcp[f]).long()
        self.xtinfo = torch.stack([f, p0, nz, torch.zeros_like(f)], 1).to(torch.int32).contiguous()
        # 128 row indices per slot (ABI 18): a one-wave column needs no index
        # loads past its head
        self.xthead = self._head_of(p0, nz, self.xrow, None, width=128)

    @staticmethod
    def _head_of(p0: torch.Tensor, nz: torch.Tensor, idx: torch.Tensor, val, width: int = 64):
        """The first `width` entries of every row of a CSR (row starts p0,
        lengths nz): indices [rows, width] int32, or {index, value bits} pairs
        [rows, width, 2] when `val` is given; zero past each row's end."""
        e = torch.arange(width, device=p0.device)
        ok = e[None, :] < nz[:, None]
        pos = torch.where(ok, p0[:, None] + e[None, :], torch.zeros_like(p0)[:, None])
        if idx.numel() == 0:
            cols = torch.zeros(pos.shape, dtype=torch.int32, device=p0.device)
            vals = torch.zeros(pos.shape, dtype=torch.float32, device=p0.device)
        else:
            cols = torch.where(ok, idx[pos].to(torch.int32), 0)
            vals = torch.where(ok, val[pos], 0.0) if val is not None else None
        if val is None:
            return cols.to(torch.int32).contiguous()
        return torch.stack([cols.to(torch.int32), vals.to(torch.float32).view(torch.int32)], 2).contiguous()

    def _xt_split(self, xcsc: torch.Tensor, d: torch.Tensor, fwd_off: int):
        """Long X columns: run the column products as xt_splits partial ranges
        (lds_engine_xt_partials) and return xt_adam's (xt_part, xt_splits,
        column order, heavy count)."""
        if self.xt_splits <= 1:
            return 0, 0, nat.ptr(self.xt_order), self.xt_heavy
        nat.call("lds_engine_xt_partials", nat.ptr(self.xcp), nat.ptr(self.xrow), nat.ptr(xcsc), self.fin,
                 nat.ptr(d), self.seed, self.tag_x, nat.ptr(self.scalars), fwd_off, 0, self.keep, self.scale,
                 self.xt_splits, nat.ptr(self.xt_part), self.btx, self._stream())
        return nat.ptr(self.xt_part), self.xt_splits, nat.ptr(self.xt_order), 0

    def _adam_args(self, mode: int, t: int, first: int = 0):
        """Trailing Adam arguments of lds_engine_final / lds_engine_xt_adam.
        mode 1: forward of inner step t; mode 2: reverse of inner step t."""
        P = nat.ptr
        if mode == 0:
            return (0, 0) + (0,) * 11 + (0, 0, self.n_wd)
        if mode == 1:
            ws = (P(self.w[t]), P(self.m[t]), P(self.v[t]), P(self.w[t + 1]), P(self.m[t + 1]), P(self.v[t + 1]),
                  P(self.gp[t]), 0, 0, 0, 0)
        else:
            ws = (0, 0, 0, 0, P(self.m[t + 1]), P(self.v[t + 1]), P(self.gp[t]), P(self.wbar), P(self.mbar),
                  P(self.vbar), P(self.gbar))
        return (mode, first) + ws + (self.hyper_np.ctypes.data, P(self.adam_tab), self.n_wd)

    def _xvals(self, sl: _Slot):
        """(CSR, CSC) values of X as the slot's training forward used them."""
        if self.train_flag:
            return sl.xd_csr, sl.xd_csc
        return self.xval, self.xtval

    def _backward(self, sl: _Slot, w: torch.Tensor, gout: torch.Tensor, train: int, fwd_off: int,
                  metrics_row: torch.Tensor, outer_factors: bool, adam_mode: int, adam_t: int,
                  mask_bit: int = 0, inv_count: float = 0.0, bt2=None):
        """First-order backward into `gout` (data gradient, no weight decay),
        fused with the Adam forward of inner step adam_t (adam_mode 1) or the
        Adam reverse of inner step adam_t (adam_mode 2, hyper step).  With the
        two-hop kernels the loss layer over the rows of `mask_bit` runs here
        (lds_engine_fwd2_bwd2)."""
        st, n, c = self._stream(), self.n, self.c
        _, _, w1, _ = self._views(w)
        g = sl.g
        if outer_factors:
            base = self.t * self.kg
            (U, V, ldu), R = self._uv(), self._r_of(self.t)
        else:
            base, U, V, R, ldu = 0, 0, 0, 0, self.ldu
        rp, cl, s, el = nat.ptr(g.row_ptr), nat.ptr(g.col), nat.ptr(g.s), nat.ptr(g.ell)
        if self.two_hop and (mask_bit == 1 or self.two_hop_outer):
            nat.call("lds_engine_fwd2_bwd2", rp, cl, s, el, n, nat.ptr(self.nflag), mask_bit, nat.ptr(sl.h2),
                     nat.ptr(sl.o), nat.ptr(sl.p), nat.ptr(sl.d_o), nat.ptr(self.label), inv_count,
                     nat.ptr(sl.lossrow), nat.ptr(sl.corrrow), c, nat.ptr(sl.y0), nat.ptr(sl.dh2), nat.ptr(sl.dy0),
                     nat.ptr(w1), self.seed, self.tag_h, nat.ptr(self.scalars), fwd_off, train, self.keep,
                     self.scale, U, V, ldu, R, base + HID, self.cw, 1, nat.ptr(sl.dmask),
                     self.bt2 if bt2 is None else bt2, st)
        else:
            nat.call("lds_engine_bwd_layer2", rp, cl, s, el, n, nat.ptr(sl.d_o), nat.ptr(sl.y0), nat.ptr(sl.dh2),
                     nat.ptr(sl.dy0), nat.ptr(w1), c, self.seed, self.tag_h, nat.ptr(self.scalars), fwd_off, train,
                     self.keep, self.scale, nat.ptr(sl.o), nat.ptr(sl.h2), U, V, ldu, R, base + HID, self.cw,
                     1, nat.ptr(sl.dmask), self._agg(g, sl.d_o), self.bt, st)
        # dH0 + first stage of gW1 = dH2ᵀ H1d, gb0 = Σ dH0, gb1 = Σ dH2, loss / correct
        nat.call("lds_engine_bwd1_reduce", rp, cl, s, el, n, nat.ptr(sl.dy0), nat.ptr(sl.dh0), nat.ptr(sl.y0),
                 nat.ptr(sl.h0), U, V, ldu, R, base, nat.ptr(sl.dh2), nat.ptr(sl.h1d), nat.ptr(sl.lossrow),
                 nat.ptr(sl.corrrow), c, nat.ptr(self.partials), self._agg(g, sl.dy0), self.bt, st)
        first = 1 if adam_mode == 2 else 0
        adam = self._adam_args(adam_mode, adam_t, first)
        # W0 part (Xdᵀ dH0) and the final stage of the reduction, one launch
        xcsc = self._xvals(sl)[1]
        nat.call("lds_engine_xt_adam", nat.ptr(self.xcp), nat.ptr(self.xrow), nat.ptr(xcsc),
                 self.fin, nat.ptr(sl.dh0), nat.ptr(gout), 0, self.seed, self.tag_x, nat.ptr(self.scalars), fwd_off,
                 0, self.keep, self.scale, nat.ptr(self.partials), self.nred, c, self.off_b0, self.off_w1,
                 self.off_b1, nat.ptr(metrics_row), *adam, adam_t, *self._xt_split(xcsc, sl.dh0, fwd_off),
                 nat.ptr(self.xtinfo), nat.ptr(self.xthead), self.xt_n1, self.xt_n2, self.btx, st)

    # ----------------------------------------------------------------- steps
    def _sample_batch(self, count: int):
        """Draw the window's `count` graphs in one batched launch set; graph g
        takes draw counter (pending + g), exactly the counter the step-by-step
        path would give it."""
        self._flush_fill()
        gb = self.gbatch
        if self._prefetched:  # bits + degrees drawn by the last hyper step (lds_theta_grad_sgd_draw)
            fill = (nat.ptr(gb.bits), self.words, nat.ptr(gb.deg), count * self.S, nat.ptr(gb.row_ptr),
                    self._col_arg(gb.col), max(self.cap, 1), nat.ptr(gb.s), nat.ptr(gb.ell), nat.ptr(self.nflag))
            if self.fuse_fill and not self.long_rows:
                # deferred: the first inner step's X product launches it (lds_engine_fill_x_linear)
                self._pending_fill = fill
            else:
                nat.call("lds_sample_fill_csr", fill[0], self.n, *fill[1:], self._err_ptr(), self._stream())
            self._prefetched = False
        elif self.shards is not None:
            self._sharded_draw(gb.bits, gb.deg, gb.s, (gb.row_ptr, gb.col, gb.ell), count, self.pending_graph)
        elif self.async_draw and count > 1 and not self.long_rows:
            # graph 0 on the main stream; graphs 1 .. count-1 on the side stream,
            # beside inner step 0 (joined before step 1: _join_draw)
            self._draw_range(0, 1, self._stream())
            side = self.side
            side.wait_stream(torch.cuda.current_stream(self.dev))
            self._draw_range(1, count - 1, side.cuda_stream)
            self._draw_pending = True
        else:
            self._draw_range(0, count, self._stream())
        self._ws_clean = False
        self._block_ptrs(gb.graphs[:count])

    def _flush_fill(self):
        """A deferred window fill runs now (something else needs the graphs
        before the first X product)."""
        if self._pending_fill is not None:
            f, self._pending_fill = self._pending_fill, None
            nat.call("lds_sample_fill_csr", f[0], self.n, *f[1:], self._err_ptr(), self._stream())

    def _draw_range(self, g0: int, count: int, stream: int):
        """Graphs g0 .. g0 + count - 1 of the window (all samples), counters
        pending + g0 + g, into the batch's graph slots g0 + g."""
        gb, S, P = self.gbatch, self.S, nat.ptr

        def at(t: torch.Tensor) -> int:  # graph g0 of a [count][S][...] batch array
            return P(t) + g0 * t[0].numel() * t.element_size()
        nat.call("lds_sample_graphs_multi", P(self.theta), self.n, self.seed, self.tag_graph, 1, P(self.scalars),
                 self.pending_graph + g0, count, S, at(gb.bits), self.words, at(gb.deg), at(gb.row_ptr),
                 at(gb.col) if not self.bitmask_agg else 0, max(self.cap, 1), at(gb.s), at(gb.ell),
                 P(self.nflag), 1 if self._ws_clean else 0, self._err_ptr(), stream)

    def _join_draw(self):
        """The window's later graphs (drawn on the side stream) are complete
        before their first use."""
        if self._draw_pending:
            torch.cuda.current_stream(self.dev).wait_stream(self.side)
            self._draw_pending = False

    def discard_prefetched_draws(self):
        """Forget graphs a hyper step drew for the next window (θ about to be
        rewritten from outside the engine); the next window draws its own."""
        self._drop_prefetch()

    def _drop_prefetch(self):
        """A draw or counter use outside a window replay: the prefetched
        graphs are discarded (the next window draws its own with the counters
        it then finds); gbatch.deg holds their degrees, so it is cleared first."""
        if self._prefetched:
            self._prefetched = False
            self._ws_clean = False

    def _planes_window(self, T: int, grad_reducer) -> bool:
        """This hyper step assembles dθ with the direct-staged form
        (lds_theta_grad_direct: the factor producers write split-bf16 planes,
        the θ-grad kernel stages them by direct global -> LDS loads): one
        sample, a full window (its columns are the same every window, so no
        stale plane columns), no model outer step, no per-draw θ, and the form "bf16x3-direct" or the by-shape
        default where the 128-tile grid is at most one tile per CU (Cora-sized
        graphs; MI355X: 55.0 vs 62.4 µs with the next window's draw,
        profiles/r03_theta_direct_forms.jsonl).  With an exchange (round 5) it
        assembles dθ alone (mode 0) and the SGD + draw follow the reducer.
        Same result bits as the fp32-operand forms."""
        form = self._form_name()
        if not self.uv_planes or self.S != 1 or T != self.tau:
            return False
        if self.outer_update is not None or self.theta_fn is not None or self.split_theta_grad or \
                self.shards is not None:
            return False
        nb = (self.n + 127) // 128
        return form == "bf16x3-direct" or (form == "bf16x3" and nb * (nb + 1) // 2 <= 256)

    def _uv(self):
        """(U, V, ld) of the factor producers' launches: fp32 rows (ld > 0) or,
        in a planes window, the split planes (ld = -row tiles)."""
        if self._planes_now:
            if self.Up is None:
                ne = int(nat.lib.lds_planes_t128_elems(self.n, self.ktot))
                self.Up = torch.zeros(ne, dtype=torch.int16, device=self.dev)
                self.Vp = torch.zeros(ne, dtype=torch.int16, device=self.dev)
            return nat.ptr(self.Up), nat.ptr(self.Vp), -((self.n + 127) // 128)
        return nat.ptr(self.U), nat.ptr(self.V), self.ldu

    def _prefetch_ok(self, T: int, k0: int, exchange: bool = False, check_flag: bool = True) -> bool:
        """The next window's draw can ride in this hyper step: plain LDS θ, a
        full window; with an exchange (dθ all-reduced before the SGD step) in
        the SGD + clamp pass (lds_sgd_sample_graphs, any S, CSR graphs), else
        in the θ-grad kernel: single sample, a split-bf16 form with aligned
        operands (lds_theta_grad_sgd_draw: the 64-tile form at Cora-sized
        shapes, the 128-tile form at large n, where the bitmask-aggregated
        window then needs only s from the drawn degrees)."""
        if not ((self.prefetch_draw or not check_flag) and self.theta_fn is None and self.outer_update is None
                and T == self.tau and self.gbatch.count == self.tau + 1):
            return False
        if exchange:
            return not self.bitmask_agg
        if self.S != 1 or self._form_name() == "fp32":
            return False
        if self._planes_now:
            return True
        return self.ldk % 4 == 0 and k0 % 8 == 0 and nat.ptr(self.U) % 16 == 0 and nat.ptr(self.V) % 16 == 0

    def inner_step(self, presampled: bool = False):
        """One InnerProblemTrainer.train_step (sample + forward + backward +
        differentiable Adam), recorded on the tape.  Metrics stay on device
        (`metrics[t]` = [Σ NLL over train rows, #correct])."""
        t = self.t
        if t >= len(self.slots):
            self._grow(t + 1)
            self.tau = t + 1
            self._alloc_factors()
            self.metrics = torch.zeros((self.tau + 1, self.S, 2), dtype=torch.float32, device=self.dev)
            self._refresh_adam_table()  # entries for the new step offsets
        sl = self.slots[t]
        if t > 0:
            self._flush_fill()
            self._join_draw()
        if self.theta_fn is not None:
            assert not presampled
            self._sample_per_draw(sl.g, t)
        elif presampled:
            self.pending_graph += 1
        else:
            self._sample(sl.g)
        fwd_off = self.pending_fwd
        self._fwd_of[t] = fwd_off
        self._forward(sl, self.w[t], self.train_mask, self.inv_train, self.train_flag, fwd_off,
                      loss_in_backward=True)
        self._backward(sl, self.w[t], self.g, self.train_flag, fwd_off, self.metrics[t], False, 1, t,
                       mask_bit=1, inv_count=self.inv_train)
        if self.train_flag:
            self.pending_fwd += 1
        self.t = t + 1
        return self.metrics[t]

    def hyper_step(self, grad_reducer=None, presampled: bool = False):
        """OuterProblemTrainer.train_step + both detaches.  Returns the device
        metrics row [Σ NLL over opt rows, #correct]."""
        st, n, c = self._stream(), self.n, self.c
        drew = False
        if not presampled:
            self._drop_prefetch()
        if self.outer_update is not None:
            if self.S > 1:
                raise NotImplementedError("outer_update (θ as a function of model parameters) is single-sample")
            if grad_reducer is None:  # the model's outer step takes the reducer's place (capture: the split point)
                grad_reducer = self.outer_update
        elif grad_reducer is None:
            grad_reducer = self.grad_reducer  # replicas over ranks: dθ → all-reduce → SGD (never fused)
        T = self.t
        if T * self.kg + HID + self.cw > self.ldk:
            self._alloc_factors()
        self._planes_now = self._planes_window(T, grad_reducer)
        out = self.outer
        self._flush_fill()
        self._join_draw()
        if self.theta_fn is not None:
            assert not presampled
            self._sample_per_draw(out.g, T)
        elif presampled:
            self.pending_graph += 1
        else:
            self._sample(out.g)
        fwd_off = self.pending_fwd
        self._forward(out, self.w[T], self.opt_mask, self.inv_opt, self.train_flag, fwd_off,
                      loss_in_backward=self.two_hop_outer)
        # R is assigned by the outer layer-2 backward (first emitter); the
        # Adam reverse of step T-1 starts from zero m̄ / v̄ (`first`)
        self._backward(out, self.w[T], self.wbar, self.train_flag, fwd_off, self.metrics[self.tau], True,
                       2 if T else 0, T - 1 if T else 0, mask_bit=2, inv_count=self.inv_opt)
        if self.train_flag:
            self.pending_fwd += 1
        if self.theta_fn is not None:
            return self._hyper_tail_per_draw(T, grad_reducer)
        split = self.split_theta_grad and T > 0
        if split and self.S > 1:
            raise NotImplementedError("split θ-grad assembly is single-sample only")
        if split:  # outer graph's columns: first chunk of dθ, beside reverse step T-1
            self._theta_chunk(T * self.kg, HID + self.cw, accumulate=0)
        for t in range(T - 1, -1, -1):
            self._reverse_step(t)
            if split and t > 0:  # graph t's columns are final: its chunk runs beside step t-1
                self._theta_chunk(t * self.kg, self.kg, accumulate=1)
        if split:
            torch.cuda.current_stream(self.dev).wait_stream(self.side)
            k0 = self.kg  # the last chunk (graph 0) + R on the main stream
        else:
            k0 = T * self.kg + HID + self.cw
        if self.shards is not None:  # band-sharded replicas: the exchange is in the update itself
            self._sharded_update(k0)
        elif self.S > 1:
            drew = self._assemble_samples(k0, grad_reducer, presampled)
        elif grad_reducer is None:  # dθ assembly (last chunk) fused with SGD + clamp
            if split:
                nat.call("lds_theta_grad_sgd_accum", nat.ptr(self.U), nat.ptr(self.V), self.ldk, k0,
                         nat.ptr(self.R), 1, 1, nat.ptr(self.theta), n, nat.ptr(self.grad), nat.ptr(self.scalars), self._form(), st)
            elif self._planes_now:  # direct-staged form on the planes; + the next window's draw when prefetching
                graphs, bits, deg = 0, 0, 0
                if presampled and self._prefetch_ok(T, k0):
                    if self._deg_next is None:
                        self._deg_next = torch.zeros_like(self.gbatch.deg)
                    graphs = self.gbatch.count
                    bits, deg = nat.ptr(self.gbatch.bits), nat.ptr(self._deg_next)
                    drew = True
                nat.call("lds_theta_grad_direct", nat.ptr(self.Up), nat.ptr(self.Vp), k0, nat.ptr(self.R), 1, 1, 1,
                         nat.ptr(self.theta), n, nat.ptr(self.grad) if self.keep_grad else 0, 2,
                         nat.ptr(self.scalars), 1.0, self.seed, self.tag_graph, nat.ptr(self.scalars),
                         self.pending_graph, graphs, bits, self.words, deg, st)
            elif presampled and self._prefetch_ok(T, k0):  # + the next window's draw, from the θ written here
                if self._deg_next is None:
                    self._deg_next = torch.zeros_like(self.gbatch.deg)
                gb = self.gbatch
                nat.call("lds_theta_grad_sgd_draw", nat.ptr(self.U), nat.ptr(self.V), self.ldk, k0, nat.ptr(self.R),
                         1, 1, nat.ptr(self.theta), n, nat.ptr(self.grad) if self.keep_grad else 0,
                         nat.ptr(self.scalars), self.seed, self.tag_graph, nat.ptr(self.scalars), self.pending_graph,
                         gb.count, nat.ptr(gb.bits), self.words, nat.ptr(self._deg_next),
                         self._form(), st)
                drew = True
            else:
                nat.call("lds_theta_grad_sgd", nat.ptr(self.U), nat.ptr(self.V), self.ldk, k0, nat.ptr(self.R), 1,
                         1, nat.ptr(self.theta), n, nat.ptr(self.grad) if self.keep_grad else 0,
                         nat.ptr(self.scalars), self._form(), st)
        else:  # replicas: dθ, all-reduce (mean), then the identical update everywhere
            pre = self._prescale(grad_reducer) if self._planes_now else None
            if self._planes_now:  # the direct-staged form, dθ only (mode 0; no draw: that follows the exchange)
                nat.call("lds_theta_grad_direct", nat.ptr(self.Up), nat.ptr(self.Vp), k0, nat.ptr(self.R), 1, 1, 1,
                         nat.ptr(self.theta), n, nat.ptr(self.grad), 0, nat.ptr(self.scalars),
                         1.0 / pre if pre else 1.0, self.seed, self.tag_graph, nat.ptr(self.scalars),
                         self.pending_graph, 0, 0, self.words, 0, st)
            else:
                nat.call("lds_theta_grad", nat.ptr(self.U), nat.ptr(self.V), self.ldk, k0, nat.ptr(self.R), 1, 1,
                         nat.ptr(self.theta), n, nat.ptr(self.grad), 1 if split else 0, self._form(), st)
            if pre:  # dθ already scaled by 1/world: the exchange is the all-reduce SUM alone
                grad_reducer(self.grad, prescaled=True)
            else:
                grad_reducer(self.grad)  # with outer_update: the model's optimizer step, which rewrites θ
            if self.outer_update is None:
                drew = self._sgd_step(T, k0, presampled)
        # detach: the window restarts from the latest weights / Adam state
        # (a prefetched draw's degrees move into gbatch.deg for the next fill)
        P = nat.ptr
        wmv = (P(self.w[T]), P(self.m[T]), P(self.v[T])) if T else (0, 0, 0)
        nat.call("lds_engine_end_window", self.np, *wmv, P(self.w[0]), P(self.m[0]), P(self.v[0]),
                 P(self.scalars), self.pending_graph, self.pending_fwd, T, 1, P(self.betas_dev), P(self.adam_tab),
                 self._tab_count(), P(self.gbatch.deg), P(self._deg_next) if drew else 0, self.gbatch.deg.numel(),
                 self.bt, st)
        self._prefetched = drew
        self._ws_clean = not drew
        self._planes_now = False
        self.pending_graph = 0
        self.pending_fwd = 0
        self.t = 0
        return self.metrics[self.tau]

    def _sgd_step(self, T: int, k0: int, presampled: bool) -> bool:
        """SGD + clamp of θ after the exchange; with prefetched draws fused
        with the next window's draw (lds_sgd_sample_graphs).  True if it drew."""
        st, P = self._stream(), nat.ptr
        if presampled and self._prefetch_ok(T, k0, exchange=True):
            if self._deg_next is None:
                self._deg_next = torch.zeros_like(self.gbatch.deg)
            gb = self.gbatch
            nat.call("lds_sgd_sample_graphs", P(self.theta), P(self.grad), P(self.scalars), self.n, self.seed,
                     self.tag_graph, 1, self.pending_graph, gb.count, self.S, P(gb.bits), self.words,
                     P(self._deg_next), P(self._sgd_tiles) if self.sgd_draw_split else 0, st)
            if self.sgd_draw_split and not self._sgd_tiles_checked and not torch.cuda.is_current_stream_capturing():
                # the per-tile counters must come back to zero (their protocol
                # assumes zero on entry); checked once, on the first eager call
                # (round-5 ADVICE); later stale counters set
                # LDS_DEVERR_SGD_TILE_COUNTER in the device error word
                self._sgd_tiles_checked = True
                if int(torch.count_nonzero(self._sgd_tiles).item()) != 0:
                    nat.raise_device_error(nat.DEVERR_SGD_TILE_COUNTER, "LdsEngine (SGD + draw tile counters)")
            return True
        nat.call("lds_engine_sgd_clamp", P(self.theta), P(self.grad), self.theta.numel(), P(self.scalars), st)
        return False

    def _assemble_samples(self, k0: int, grad_reducer, presampled: bool = False) -> bool:
        """Mean hypergradient of the S replica samples: one rank-(S·ldk)
        update over the side-by-side factor blocks (columns past k0 of each
        block zeroed first), R summed over the S stacked rows, gscale = 1/S;
        fused with SGD + clamp, or (replicas over ranks) dθ → reducer → SGD."""
        st, n, S = self._stream(), self.n, self.S
        if k0 < self.ldk:  # stale columns of a longer earlier window
            self.U.view(n, S, self.ldk)[:, :, k0:].zero_()
            self.V.view(n, S, self.ldk)[:, :, k0:].zero_()
        P = nat.ptr
        gs = float(np.float32(1.0) / np.float32(S))
        pre = self._prescale(grad_reducer) if grad_reducer is not None else None
        if pre:  # × 2^-k: exact, the same bits as dividing the summed dθ by world
            gs = float(np.float32(gs) / np.float32(pre))
        if grad_reducer is None:
            nat.call("lds_theta_grad_ex", P(self.U), P(self.V), self.ldu, self.ldu, P(self.R), 1, n, S,
                     P(self.theta), n, P(self.grad) if self.keep_grad else 0, 2, P(self.scalars), gs, self._form(), st)
        else:
            nat.call("lds_theta_grad_ex", P(self.U), P(self.V), self.ldu, self.ldu, P(self.R), 1, n, S,
                     P(self.theta), n, P(self.grad), 0, 0, gs, self._form(), st)
            if pre:
                grad_reducer(self.grad, prescaled=True)
            else:
                grad_reducer(self.grad)
            return self._sgd_step(self.tau if presampled else -1, k0, presampled)
        return False

    # ------------------------------------------------ band-sharded replicas
    def set_band_shards(self, shards) -> None:
        """Run this long-row engine as rank `shards.rank` of band-sharded
        replicas (ldsgnn.replicas.BandShards; BASELINE config 5 at N > 1,
        DESIGN §5b): one replica per rank (replica = rank), θ current only in
        this rank's row band between sync_theta() calls.  Every hyper step
        all-gathers the ranks' θ-gradient factors and updates the band
        (lds_theta_grad_band: the mean hypergradient, fused SGD + clamp);
        every draw takes the band's rows of every replica's graphs
        (lds_sample_band_bits), exchanges them (all-to-all) and completes
        this replica's graphs (lds_bitmask_mirror_degree).  Windows run
        eagerly (run_window).  With world 1 the results are bit-identical to
        the engine's own exchange path (dθ, then SGD + clamp)."""
        from .rng import TAG_GRAPH as _TG
        if not self.long_rows or self.S != 1:
            raise NotImplementedError("band-sharded replicas: the long-row engine, one sample per rank")
        if self.theta_fn is not None or self.outer_update is not None:
            raise NotImplementedError("band-sharded replicas: plain LDS θ")
        if self.tag_graph != tag_for(_TG, shards.rank):
            raise ValueError("band-sharded replicas: this engine's replica must equal its rank "
                             "(ldsgnn.rng.manual_seed(seed, replica=rank))")
        if shards.n != self.n:
            raise ValueError("band-sharded replicas: bands built for another n")
        self._drop_prefetch()
        self.prefetch_draw = False
        self.shards = shards
        self._theta_whole = True

    def sync_theta(self) -> None:
        """Every rank's band of θ into every rank's copy (all-gather): the
        full, identical θ on all ranks (evaluation, checkpoints, the drop-in
        model's probs)."""
        if self.shards is not None:
            self.shards.gather_rows(self.theta.view(-1), self.n)
            self._theta_whole = True

    def _sharded_update(self, k0: int) -> None:
        """The mean hypergradient of all ranks' replicas on this rank's band,
        fused with SGD + clamp there: every rank's factors all-gathered and
        side by side (replica q in columns [q·ldk, (q+1)·ldk)), R stacked,
        gscale = 1/world — the arithmetic of a batched engine's rank-(S·K)
        assembly.  θ.grad (if kept) holds the band's dθ."""
        st, n, P, sh = self._stream(), self.n, nat.ptr, self.shards
        if k0 < self.ldu:  # stale columns of a longer earlier window
            self.U[:, k0:].zero_()
            self.V[:, k0:].zero_()
        N = sh.world
        if not sh._skip:
            uc = sh.all_gather(self.U).permute(1, 0, 2).contiguous()  # [n, N, ldk]
            vc = sh.all_gather(self.V).permute(1, 0, 2).contiguous()
            rg = sh.all_gather(self.R[0])  # [N, n]
        else:
            uc, vc, rg = self.U, self.V, self.R
        ld = N * self.ldu
        gs = float(np.float32(1.0) / np.float32(N))
        row0, row1 = sh.band
        nat.call("lds_theta_grad_band", P(uc), P(vc), ld, ld, P(rg), 1, n, N, P(self.theta), n,
                 P(self.grad) if self.keep_grad else 0, 2, P(self.scalars), gs, row0, row1, st)
        self._theta_whole = N == 1

    def _sharded_draw(self, bits: torch.Tensor, deg: torch.Tensor, s: torch.Tensor, csr, count: int,
                      counter_off: int) -> None:
        """`count` graphs of this rank's replica (draw counters counter_off + g)
        into bits [count, 1, n, words] with their degrees (deg [count, 1, wsi])
        and s, and (CSR modes) row_ptr / col / ELL: this rank draws its band's
        rows of EVERY replica's graphs, the bands meet at their owners
        (all-to-all), the owner mirrors its graphs' lower triangle."""
        from .rng import TAG_GRAPH as _TG
        st, n, W, P, sh = self._stream(), self.n, self.words, nat.ptr, self.shards
        N = sh.world
        row0, row1 = sh.band
        need = count * N * n * W
        if self._allbits is None or self._allbits.numel() < need:
            # zeroed once: a row's padding word past ceil(n/64) (words is even) is never drawn
            self._allbits = torch.zeros(need, dtype=torch.int64, device=self.dev)
        ab = self._allbits[:need].view(count, N, n, W)
        nat.call("lds_sample_band_bits", P(self.theta), n, self.seed, tag_for(_TG, 0), 1, P(self.scalars),
                 counter_off, count, N, row0, row1, P(ab), W, st)
        sh.exchange_rows(ab, bits.view(count, n, W))
        nat.call("lds_bitmask_mirror_degree", P(bits), n, W, count, P(deg), P(s), st)
        self._ws_clean = False
        if not self.bitmask_agg:  # CSR / s / ELL from the completed bits and their degree counts
            row_ptr, col, ell = csr
            nat.call("lds_sample_fill_csr", P(bits), n, W, P(deg), count, P(row_ptr), P(col), max(self.cap, 1),
                     P(s), P(ell), P(self.nflag), self._err_ptr(), st)

    @staticmethod
    def _prescale(grad_reducer):
        """World size w when `grad_reducer` takes a dθ the assembly scaled by
        1/w (its `prescale` attribute, ldsgnn.fused for replicas.allreduce_mean
        over a power-of-two world): the exchange is then the all-reduce SUM
        alone, with no division pass over θ.grad.  None: an ordinary reducer."""
        f = getattr(grad_reducer, "prescale", None)
        w = f() if callable(f) else f
        return int(w) if w else None

    def _theta_chunk(self, col0: int, k: int, accumulate: int):
        """grad (=|+=) U[:, col0:col0+k] V[...]ᵀ + V U ᵀ on the side stream, after
        everything queued so far on the main stream (no R, no clamp mask:
        the last chunk adds them)."""
        side = self.side
        side.wait_stream(torch.cuda.current_stream(self.dev))
        off = 4 * col0
        nat.call("lds_theta_grad", nat.ptr(self.U) + off, nat.ptr(self.V) + off, self.ldk, k, 0, 0, 0, 0, self.n,
                 nat.ptr(self.grad), accumulate, self._form(), side.cuda_stream)

    # ------------------------------------------------------- per-draw θ
    def set_theta_fn(self, fn):
        """θ as a function of the draw: every graph of a window is sampled
        from its own θ_t = fn(counter_t), counter_t the forward counter the
        model's own forward takes right before the draw (a GAE proposal GCN
        with dropout: src/models/graph.py:167-186 runs once per sample()).  The
        hyper step then assembles one dθ_t per draw (its factor columns and its
        own R row) and hands the stack [T + 1, n(n+1)/2] to the reducer
        (outer_update), which takes each through its own P_t.  Single sample,
        eager windows."""
        self._drop_prefetch()
        if self.S != 1:
            raise NotImplementedError("per-draw θ is single-sample")
        self.theta_fn = fn
        self.theta_counters = {}

    def detach(self):
        """InnerProblemTrainer.detach without a hyper step (a training loop
        with no graph learning, BASELINE config 1): the weights and Adam state
        of the current step become slot 0, the pending draw counters and Adam
        steps are applied on device (lds_engine_end_window with no hyper step:
        no learning-rate decay)."""
        self._drop_prefetch()
        T, P, st = self.t, nat.ptr, self._stream()
        wmv = (P(self.w[T]), P(self.m[T]), P(self.v[T])) if T else (0, 0, 0)
        nat.call("lds_engine_end_window", self.np, *wmv, P(self.w[0]), P(self.m[0]), P(self.v[0]),
                 P(self.scalars), self.pending_graph, self.pending_fwd, T, 0, P(self.betas_dev), P(self.adam_tab),
                 self._tab_count(), P(self.gbatch.deg), 0, self.gbatch.deg.numel(), self.bt, st)
        self._ws_clean = True
        self.pending_graph = 0
        self.pending_fwd = 0
        self.t = 0

    def take_forward_counter(self) -> int:
        """The next forward counter (absolute), taken by a host-side forward
        (per-draw θ: the model's statistics() in training mode)."""
        c = int(self._i32[1].item()) + self.pending_fwd
        self.pending_fwd += 1
        return c

    def _per_draw_bufs(self, count: int):
        tri = self.theta.numel()
        if getattr(self, "theta_g", None) is None or self.theta_g.size(0) < count:
            self.theta_g = torch.zeros((count, tri), dtype=torch.float32, device=self.dev)
            self.grad_g = torch.zeros((count, tri), dtype=torch.float32, device=self.dev)
            self.Rg = torch.zeros((count, self.n), dtype=torch.float32, device=self.dev)

    def _sample_per_draw(self, g: _Graph, slot: int):
        """θ_slot = theta_fn(absolute forward counter), then the draw from it;
        the model's forward takes that counter (pending_fwd += 1)."""
        self._drop_prefetch()
        self._per_draw_bufs(max(slot + 1, self.tau + 1))
        c = int(self._i32[1].item()) + self.pending_fwd  # device counter + this window's pending forwards
        self.theta_g[slot].copy_(self.theta_fn(c))
        self.theta_counters[slot] = c
        self.pending_fwd += 1
        self._sample(g, theta=self.theta_g[slot])

    def _r_of(self, slot: int) -> int:
        """R of the factors of graph `slot`: one shared vector, or (per-draw
        θ) graph slot's own row."""
        if self.theta_fn is None:
            return nat.ptr(self.R)
        return nat.ptr(self.Rg[slot])

    def _hyper_tail_per_draw(self, T: int, grad_reducer):
        """Hyper-step tail for per-draw θ: the reverse pass (each graph's
        factors and R row), dθ_t per draw (its own columns: graph t < T at
        [t·kg, (t+1)·kg), the outer graph at [T·kg, T·kg + 16 + cw)), the
        reducer on the stack, then the detach."""
        st, n = self._stream(), self.n
        self.Rg[:T].zero_()  # inner graphs' rows accumulate (the outer row is assigned by its first emitter)
        for t in range(T - 1, -1, -1):
            self._reverse_step(t)
        for t in range(T + 1):
            k0, k = (t * self.kg, self.kg) if t < T else (T * self.kg, HID + self.cw)
            nat.call("lds_theta_grad", nat.ptr(self.U) + 4 * k0, nat.ptr(self.V) + 4 * k0, self.ldk, k,
                     nat.ptr(self.Rg[t]), 1, 1, 0, n, nat.ptr(self.grad_g[t]), 0, self._form(), st)
        grad_reducer(self.grad_g[:T + 1])
        P = nat.ptr
        wmv = (P(self.w[T]), P(self.m[T]), P(self.v[T])) if T else (0, 0, 0)
        nat.call("lds_engine_end_window", self.np, *wmv, P(self.w[0]), P(self.m[0]), P(self.v[0]),
                 P(self.scalars), self.pending_graph, self.pending_fwd, T, 1, P(self.betas_dev), P(self.adam_tab),
                 self._tab_count(), P(self.gbatch.deg), 0, self.gbatch.deg.numel(), self.bt, st)
        self._ws_clean = True
        self.pending_graph = 0
        self.pending_fwd = 0
        self.t = 0
        return self.metrics[self.tau]

    def _reverse_step(self, t: int):
        """Reverse of inner step t; gbar already holds ḡ of step t (from the
        Adam reverse fused into the previous stage).  Ends with the Adam
        reverse of step t-1 fused into the W̄ completion."""
        st, n, c = self._stream(), self.n, self.c
        sl, g = self.slots[t], self.slots[t].g
        # forward counter of inner step t within the window (per-draw θ: a
        # proposal forward precedes each classifier forward, so recorded)
        fwd_off = (self._fwd_of[t] if self.theta_fn is not None else t) if self.train_flag else 0
        gw0t, gb0, gw1, gb1 = self._views(self.gbar)
        _, _, w1, _ = self._views(self.w[t])
        base = t * self.kg
        rp, cl, s, el = nat.ptr(g.row_ptr), nat.ptr(g.col), nat.ptr(g.s), nat.ptr(g.ell)
        (U, V, ldu), R = self._uv(), self._r_of(t)
        tr = self.train_flag
        xcsr, xcsc = self._xvals(sl)  # Xd of step t (no redraw: train = 0 below)
        nat.call("lds_engine_x_linear", nat.ptr(self.xrp), nat.ptr(self.xcol), nat.ptr(xcsr), n,
                 nat.ptr(gw0t), nat.ptr(gb0), nat.ptr(self.dh0bar), self.seed, self.tag_x, nat.ptr(self.scalars),
                 fwd_off, 0, self.keep, self.scale, 0, 0, 0, nat.ptr(self.xhead), nat.ptr(self.xinfo),
                 1 if xcsr is self.xval else 0, self.btx, st)
        nat.call("lds_engine_rev_a", rp, cl, s, el, n, nat.ptr(self.dh0bar), nat.ptr(sl.dy0), nat.ptr(sl.dh0),
                 nat.ptr(sl.y0), nat.ptr(sl.h1d), nat.ptr(sl.dh2), nat.ptr(w1), nat.ptr(gw1), nat.ptr(gb1), c,
                 nat.ptr(self.dh1dbar), nat.ptr(self.dh2bar), nat.ptr(self.h1dbar), self.seed, self.tag_h,
                 nat.ptr(self.scalars), fwd_off, tr, self.keep, self.scale, U, V, ldu, R,
                 base + HID + 2 * self.cw, nat.ptr(sl.dmask), self._agg(g, self.dh0bar), self.bt, st)
        if self.two_hop:  # dŌ, Ōbar on the train rows only, H2bar from them: one launch
            nat.call("lds_engine_rev_bc", rp, cl, s, el, n, nat.ptr(self.nflag), 1, nat.ptr(self.dh2bar),
                     nat.ptr(sl.d_o), nat.ptr(sl.dh2), nat.ptr(sl.p), nat.ptr(sl.h2), nat.ptr(sl.o), self.inv_train, c,
                     nat.ptr(self.h1dbar), nat.ptr(sl.y0), nat.ptr(w1), nat.ptr(self.h2bar), nat.ptr(self.y0bar),
                     self.seed, self.tag_h, nat.ptr(self.scalars), fwd_off, tr, self.keep, self.scale, U, V,
                     ldu, R, base + HID + self.cw, base + HID, self.cw, nat.ptr(sl.dmask), self.bt2, st)
        else:
            nat.call("lds_engine_rev_b", rp, cl, s, el, n, nat.ptr(self.dh2bar), nat.ptr(sl.d_o), nat.ptr(sl.dh2),
                     nat.ptr(sl.p), nat.ptr(self.train_mask), self.inv_train, c, nat.ptr(self.obar), U, V, ldu,
                     R, base + HID + self.cw, self.cw, self._agg(g, self.dh2bar), self.bt, st)
            nat.call("lds_engine_rev_c", rp, cl, s, el, n, nat.ptr(self.obar), nat.ptr(sl.h2), nat.ptr(sl.o),
                     nat.ptr(self.h1dbar), nat.ptr(sl.y0), nat.ptr(w1), c, nat.ptr(self.h2bar), nat.ptr(self.y0bar),
                     self.seed, self.tag_h, nat.ptr(self.scalars), fwd_off, tr, self.keep, self.scale, U, V,
                     ldu, R, base + HID, self.cw, nat.ptr(sl.dmask), self._agg(g, self.obar), self.bt, st)
        # H0bar + first stage of W̄1 += dH2ᵀ dH1dbar + H2barᵀ H1d;  b̄0 += Σ H0bar;  b̄1 += Σ H2bar
        nat.call("lds_engine_rev_d_reduce", rp, cl, s, el, n, nat.ptr(self.y0bar), nat.ptr(sl.h0), nat.ptr(sl.y0),
                 nat.ptr(self.h0bar), U, V, ldu, R, base, nat.ptr(sl.dh2), nat.ptr(self.dh1dbar),
                 nat.ptr(self.h2bar), nat.ptr(sl.h1d), c, nat.ptr(self.partials), self._agg(g, self.y0bar), self.bt,
                 st)
        if t == 0:  # W̄ of the window's first weights feeds nothing (only θ is trained): no W0 products
            return
        adam = self._adam_args(2, t - 1)
        nat.call("lds_engine_xt_adam", nat.ptr(self.xcp), nat.ptr(self.xrow), nat.ptr(xcsc), self.fin,
                 nat.ptr(self.h0bar), nat.ptr(self.wbar), 1, self.seed, self.tag_x, nat.ptr(self.scalars), fwd_off,
                 0, self.keep, self.scale, nat.ptr(self.partials), self.nred, c, self.off_b0, self.off_w1,
                 self.off_b1, 0, *adam, t - 1, *self._xt_split(xcsc, self.h0bar, fwd_off), nat.ptr(self.xtinfo),
                 nat.ptr(self.xthead), self.xt_n1, self.xt_n2, self.btx, st)

    # ------------------------------------------------------------- graphs
    # ------------------------------------------------------ per-step graphs
    def _graphed(self, kind: str, fn):
        """Run fn() (inner_step or hyper_step) from a HIP graph captured for
        this exact launch sequence: the step's position and pending counter
        offsets (baked into the launch arguments), the Adam-table length and
        the buffer layout.  A key runs eagerly the first time it is seen
        (buffers grow then), is captured and replayed the second time and
        replayed after that; the host-side state the eager call would leave
        (position, pending offsets) is restored from the capture."""
        # everything the captured launches bake in: position, pending counter
        # offsets, Adam-table length, the θ-grad form, whether dθ is written,
        # and the buffer layout (last)
        key = (kind, self.t, self.pending_graph, self.pending_fwd, self.train_flag, self._tab_count(),
               self._form_name(), self.keep_grad, self.uv_planes, self._layout_version)
        cache = self._step_graphs
        stale = [k for k in cache if k[-1] != self._layout_version]
        for k in stale:  # captures over re-laid buffers never replay again: free their pools
            del cache[k]
        hit = cache.get(key)
        if hit is None:
            if key not in self._step_seen:
                self._step_seen.add(key)
                return fn()
            s = torch.cuda.Stream(self.dev)
            s.wait_stream(torch.cuda.current_stream(self.dev))
            graph = nat.new_graph()
            box, state = [], self._host_state()
            try:
                capture_into(graph, s, lambda: box.append(fn()), joins=(self.side,))
            except Exception:
                torch.cuda.current_stream(self.dev).wait_stream(s)
                self._restore_host_state(state)
                raise
            ret = box[0]
            torch.cuda.current_stream(self.dev).wait_stream(s)
            if self._layout_version != key[-1]:  # the call re-laid buffers: never replay it
                raise RuntimeError("engine buffers were re-allocated during step capture")
            nat.seal_graph(graph, f"{kind} step")
            hit = cache[key] = (graph, (self.t, self.pending_graph, self.pending_fwd), ret)
        graph, post, ret = hit
        graph.replay()
        self.t, self.pending_graph, self.pending_fwd = post
        return ret

    def inner_step_graphed(self):
        """inner_step() from a per-position HIP graph (see _graphed); the
        first step at a new position grows the tape eagerly."""
        if self.t >= len(self.slots) or self.theta_fn is not None:  # per-draw θ: host-side counters
            return self.inner_step()
        return self._graphed("inner", self.inner_step)

    def hyper_step_graphed(self):
        """hyper_step() (single replica, no reducer) from a HIP graph keyed
        by the window length."""
        if self.t * self.kg + HID + self.cw > self.ldk or self.split_theta_grad or self.outer_update is not None \
                or self.grad_reducer is not None:  # an eager exchange sits inside the step
            return self.hyper_step()
        return self._graphed("hyper", self.hyper_step)

    def run_window(self, tau: int, grad_reducer=None):
        """τ inner steps followed by the hyper step.  A full window from a
        window start draws its τ+1 graphs in one batched launch set."""
        batch = self.t == 0 and tau == self.tau and self.gbatch.count == tau + 1 and self.theta_fn is None
        if batch:
            self._sample_batch(tau + 1)
        for _ in range(tau):
            self.inner_step(presampled=batch)
        return self.hyper_step(grad_reducer=grad_reducer, presampled=batch)

    def capture_window(self, tau: int, grad_reducer=None, windows: int = 1, prefetch: bool = False,
                       capture_exchange: Optional[bool] = None):
        """Record run_window(tau) as HIP graphs (state must be at a window
        start).  Replays advance RNG counters, Adam step and lr on device.

        Without a reducer the window is ONE graph (dθ assembly fused with the
        SGD step); `windows` > 1 also records that many consecutive windows as
        one graph, which replay() uses for whole groups (the launches of every
        window are the same, so no boundary between two graph launches falls
        inside a group).  `prefetch`: each window's hyper step also draws
        the next window's graphs from the θ it writes — in the θ-grad kernel
        (lds_theta_grad_sgd_draw; single sample, 64-tile shapes) or, with a
        reducer, in the SGD + clamp pass after the exchange
        (lds_sgd_sample_graphs; any S) — so a window starts with the CSR fill
        only; the graphs of the first replayed window are drawn here,
        eagerly; ignored where neither applies.  Same draws, same counters,
        same results as windows that draw their own graphs.  The engine's
        own out-of-window draws and parameter changes discard the prefetched
        graphs; a caller that rewrites θ in place between windows calls
        discard_prefetched_draws() first.  With a reducer
        (replicas over RCCL) the window is
        split at the exchange: graph A runs up to dθ, `grad_reducer(grad)`
        runs eagerly between the replays (the collective stays outside the
        captured work), graph B applies SGD + clamp and the detach.
        `capture_exchange` (default: the reducer's own `capturable` attribute,
        which ldsgnn.replicas sets for the RCCL all-reduce): the exchange is
        captured INTO the window graph (an RCCL collective is a kernel node),
        so the window is one graph again and `windows` > 1 groups replay as
        at N = 1."""
        assert self.t == 0 and self.pending_graph == 0 and self.pending_fwd == 0
        if self.theta_fn is not None:
            raise NotImplementedError("per-draw θ (GAE proposal dropout) computes θ of each draw on the host "
                                      "side's counters: run windows eagerly")
        if tau != self.tau:
            raise ValueError(f"engine was built for tau={self.tau}; capture that window length")
        if self.shards is not None:
            raise NotImplementedError("band-sharded windows run eagerly (run_window): their exchange is two "
                                      "collectives per window around host-sized buffers")
        if windows < 1:
            raise ValueError("windows >= 1")
        if grad_reducer is None:
            grad_reducer = self.grad_reducer
        # every capture sets the flag (an earlier prefetching capture must not
        # leak into this one) and starts from the entry state its graphs
        # assume: prefetched draws present, or none and a clean degree buffer
        self.prefetch_draw = bool(prefetch) and \
            self._prefetch_ok(tau, tau * self.kg + HID + self.cw, exchange=grad_reducer is not None, check_flag=False)
        self._enter_window_state(self.prefetch_draw, tau)
        s = torch.cuda.Stream(self.dev)
        s.wait_stream(torch.cuda.current_stream(self.dev))
        if capture_exchange is None:
            cap = getattr(grad_reducer, "capturable", False)
            capture_exchange = bool(cap() if callable(cap) else cap)
        # ranks that exchange through a collective agree on every capture's
        # outcome before any graph is replayed: a rank whose capture failed
        # must not leave the others replaying a graph that waits in the
        # collective (round-5 ADVICE).  A capture-specific failure on any rank
        # moves every rank to the split graphs; an error of the window itself
        # is raised on every rank
        collective = _collective_reducer(grad_reducer)
        state = self._host_state()
        if grad_reducer is None or capture_exchange:
            graphs, err = [], None
            try:
                for w in sorted({1, windows}):
                    graph = nat.new_graph()

                    def body(w=w):
                        for _ in range(w):
                            self.run_window(tau, grad_reducer=grad_reducer)
                    # (thread-local capture errors: a collective library's own
                    # threads may touch the runtime while the window is captured)
                    capture_into(graph, s, body, error_mode="thread_local", joins=(self.side,))
                    graphs.append((w, nat.seal_graph(graph, f"{w}-window group",
                                                     exchange=grad_reducer is not None)))
            except Exception as e:  # noqa: BLE001  (agreed on, then re-raised or retried below)
                err = e
            torch.cuda.current_stream(self.dev).wait_stream(s)
            status = _capture_status(err)
            if collective:
                status = _ranks_agree(status, self.dev)
            if status == _CAPTURE_OK:
                self._graph_capture = (tuple(graphs), tau, None, self.prefetch_draw)
                return graphs[0][1]
            del graphs
            self._restore_host_state(state)
            if status == _CAPTURE_FATAL or grad_reducer is None:
                if err is not None:
                    raise err
                raise RuntimeError("capture_window: another rank failed to capture its window")
            import warnings
            warnings.warn(f"capture_window: the exchange could not be captured on every rank "
                          f"({type(err).__name__ if err is not None else 'another rank'}); "
                          "replaying split graphs around an eager exchange", RuntimeWarning)
        head, tail = nat.new_graph(), nat.new_graph()
        pool = torch.cuda.graph_pool_handle()
        open_graph = [head]

        def switch(_grad):  # the exchange point: close graph A, open graph B
            head.capture_end()
            open_graph[0] = tail
            tail.capture_begin(pool=pool)

        err = None
        with torch.cuda.stream(s):
            head.capture_begin(pool=pool)
            try:
                self.run_window(tau, grad_reducer=switch)
            except Exception as e:  # noqa: BLE001
                err = e
                _abort_capture(open_graph[0], s, (self.side,))
            if err is None:
                tail.capture_end()
        torch.cuda.current_stream(self.dev).wait_stream(s)
        if err is None:
            try:
                nat.seal_graph(head, "window (to the exchange)")
                nat.seal_graph(tail, "window (after the exchange)")
            except Exception as e:  # noqa: BLE001
                err = e
        status = _CAPTURE_OK if err is None else _CAPTURE_FATAL  # (no capture form is left to fall back to)
        if collective:
            status = _ranks_agree(status, self.dev)
        if status != _CAPTURE_OK:
            self._restore_host_state(state)
            if err is not None:
                raise err
            raise RuntimeError("capture_window: another rank failed to capture its window")
        self._graph_capture = ((head, tail), tau, grad_reducer, self.prefetch_draw)
        return head, tail

    def _host_state(self):
        """The host-side window position a capture advances (its launches do
        not run): restored when a capture fails, so the engine stays at the
        window start it was captured from."""
        return (self.t, self.pending_graph, self.pending_fwd, self._prefetched, self._ws_clean,
                self._pending_fill, self._draw_pending, self._planes_now, dict(self._fwd_of))

    def _restore_host_state(self, st) -> None:
        (self.t, self.pending_graph, self.pending_fwd, self._prefetched, self._ws_clean,
         self._pending_fill, self._draw_pending, self._planes_now, fwd_of) = st
        self._fwd_of = dict(fwd_of)

    def _enter_window_state(self, prefetched: bool, tau: int) -> None:
        """Bring the device to the window-start state a captured window
        assumes: with prefetch, the window's τ+1 graphs already drawn (bits +
        degrees; drawn here, eagerly, if a discard, an out-of-window draw or a
        non-prefetching step dropped them); without, no prefetched graphs and
        a zeroed degree workspace (the captured draw accumulates into it)."""
        if prefetched:
            if self._deg_next is None:
                self._deg_next = torch.zeros_like(self.gbatch.deg)
            if not self._prefetched:
                self._flush_fill()
                self._join_draw()
                self.gbatch.deg.zero_()
                self._prefetched = False
                self._ws_clean = True
                self._sample_batch(tau + 1)  # bits + degrees of this window's graphs
                self._join_draw()
                self._prefetched = True
                self._ws_clean = False
        else:
            if self._prefetched or not self._ws_clean:
                self.gbatch.deg.zero_()
            self._prefetched = False
            self._ws_clean = True

    def replay(self, windows: int = 1):
        graphs, tau, reducer, prefetched = self._graph_capture
        self._flush_fill()
        self._join_draw()  # an eager split draw still running on the side stream
        self._enter_window_state(prefetched, tau)
        if reducer is None:
            (_, one), (group, multi) = graphs[0], graphs[-1]
            for _ in range(windows // group):
                multi.replay()
            for _ in range(windows % group):
                one.replay()
            return
        head, tail = graphs
        for _ in range(windows):
            head.replay()
            reducer(self.grad)
            tail.replay()

    # ------------------------------------------------------------ metrics
    def _err_ptr(self) -> int:
        """Address of the device error word (EngineScalars.error) the graph
        fills report into (include/ldsgnn.h LDS_DEVERR_*)."""
        return nat.ptr(self.scalars) + 32

    def check_device_error(self) -> None:
        """Raise nat.DeviceError if a kernel set the device error word since
        the last check (host sync); the word is cleared first, so the engine
        can be reset and reused.  Every host read of results (metrics,
        scalars, empirical_mean) checks it."""
        word = int(self._err.item())
        if word:
            self._err.zero_()
            nat.raise_device_error(word & 0xFFFFFFFF, "LdsEngine")

    def inner_metrics(self, t: int):
        """(loss, acc) of inner step t of the last window, averaged over the
        replica samples (host sync)."""
        self.check_device_error()
        row = self.metrics[t].double().mean(0).cpu()
        return float(row[0]) * self.inv_train, float(row[1]) * self.inv_train

    def outer_metrics(self):
        self.check_device_error()
        row = self.metrics[self.tau].double().mean(0).cpu()
        return float(row[0]) * self.inv_opt, float(row[1]) * self.inv_opt

    def scalars_host(self):
        self.check_device_error()
        i = self._i32.cpu().tolist()
        f = self._f64.cpu().tolist()
        return dict(graph_ctr=i[0], fwd_ctr=i[1], adam_step=i[2], hyper_steps=i[3], outer_lr=f[0], lr_decay=f[1])

    def sampled_nnz(self) -> int:
        """Stored entries (self-loops included) of the last window's outer
        graph, sample 0 (host sync).  Bitmask mode after a prefetching hyper
        step: the bits already hold the next window's graphs, so this counts
        the next window's outer graph."""
        if self.bitmask_agg:  # no CSR: count the set bits (end_window clears the degrees)
            return int(_popcount(self.gbatch.bits[self.tau, 0]))
        return int(self.gbatch.row_ptr[self.tau, 0, self.n].item())

    def sampled_nnz_mean(self) -> float:
        """Mean stored entries per sampled graph over the last batched window's
        τ+1 graphs and replica samples (host sync)."""
        if self.bitmask_agg:
            tot = sum(_popcount(self.gbatch.bits[g, b]) for g in range(self.gbatch.count) for b in range(self.S))
        else:
            tot = float(self.gbatch.row_ptr[:, :, self.n].double().sum().item())
        return float(tot) / (self.gbatch.count * self.S)

    @staticmethod
    def window_columns(tau: int, c: int) -> int:
        cw = (c + 3) & ~3
        return tau * (2 * HID + 2 * cw) + HID + cw

    def flops_theta_grad(self, tau: int) -> float:
        """Algorithmic flops of one window's assembly (S blocks of ldk columns
        when S > 1: the padded columns are multiplied too)."""
        k = self.window_columns(tau, self.c) if self.S == 1 else self.S * self.ldk
        return 4.0 * k * (self.n * (self.n + 1) // 2)

