"""Monte-Carlo sample parallelism across GPUs.

Graph samples are independent: every rank runs its own inner chain (own GCN
weights, Adam state and keyed RNG stream: replica = rank) and produces its own
θ-gradient per hyper step.  The only exchange is one all-reduce (mean) of
θ.grad over RCCL/xGMI per hyper step; every rank then applies the identical
SGD + clamp, so θ stays replicated without a broadcast.  One rank = the
reference exactly.

Under the nccl (= RCCL) backend the all-reduce is graph-capturable: the fused
engine then captures it INTO the replayed window graph
(LdsEngine.capture_window reads the reducer's `capturable` attribute), so a
rank replays whole groups of windows as at N = 1 instead of two graphs per
window around an eager collective.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist


def _group_up() -> bool:
    return dist.is_available() and dist.is_initialized()


def exchange_capturable() -> bool:
    """The exchange can be captured into a HIP graph: no process group (no
    collective at all), or the nccl backend (an RCCL kernel on the capture
    stream).  gloo copies through the host: never captured."""
    if not _group_up():
        return True
    return dist.get_backend() == "nccl"


def allreduce_mean(model: torch.nn.Module) -> None:
    """grad_reducer for OuterProblemTrainer: θ.grad <- mean over ranks (SUM,
    then ÷ world: for the power-of-two world sizes of a node this equals
    scaling each rank's gradient by 1/world exactly)."""
    if not _group_up() or dist.get_world_size() == 1:
        return
    world = dist.get_world_size()
    for p in model.parameters():
        if p.grad is not None:
            dist.all_reduce(p.grad, op=dist.ReduceOp.SUM)
            p.grad.div_(world)


allreduce_mean.capturable = exchange_capturable


def mean_prescale():
    """World size when the mean over ranks may be taken as a SUM of
    gradients each rank has already scaled by 1/world: a process group of
    more than one rank whose size is a power of two (scaling by 2^-k commutes
    with fp32 rounding, so Σ_r (g_r / world) is bit for bit (Σ_r g_r) / world,
    barring subnormals: entries near FLT_MIN may differ by up to
    world · 2^-149, world subnormal ulps).  None otherwise (sum, then divide)."""
    if not _group_up():
        return None
    world = dist.get_world_size()
    return world if world > 1 and world & (world - 1) == 0 else None


def allreduce_sum_(grad: torch.Tensor) -> None:
    """The exchange of a prescaled gradient (mean_prescale): one all-reduce
    SUM, no division pass over θ.grad."""
    if _group_up() and dist.get_world_size() > 1:
        dist.all_reduce(grad, op=dist.ReduceOp.SUM)


def allreduce_mean_always(model: torch.nn.Module) -> None:
    """allreduce_mean that runs the collective at world size 1 too (the
    world-size-1 RCCL rehearsal on one GPU: the same launches as N > 1)."""
    world = dist.get_world_size()
    for p in model.parameters():
        if p.grad is not None:
            dist.all_reduce(p.grad, op=dist.ReduceOp.SUM)
            p.grad.div_(world)


allreduce_mean_always.capturable = exchange_capturable


def collective_capture_probe(device: torch.device) -> bool:
    """Whether every rank can capture an all-reduce into a HIP graph and
    replay it correctly.  Each rank captures a small all-reduce; the ranks
    agree on the outcome with an eager all-reduce BEFORE any replay (a rank
    that failed must not leave the others waiting inside a replayed
    collective), then replay once, check the sum and agree again.  False
    without the nccl backend."""
    if not _group_up() or not exchange_capturable():
        return False
    world = dist.get_world_size()
    ok = True
    x = torch.ones(64, dtype=torch.float32, device=device)
    graph = None
    try:
        graph = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(device)
        s.wait_stream(torch.cuda.current_stream(device))
        with torch.cuda.stream(s):
            with torch.cuda.graph(graph, stream=s, capture_error_mode="thread_local"):
                dist.all_reduce(x, op=dist.ReduceOp.SUM)
        torch.cuda.current_stream(device).wait_stream(s)
    except Exception:  # noqa: BLE001  (any capture failure means: do not capture)
        ok = False

    def agree(flag: bool) -> bool:
        t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(int(t.item()))

    if not agree(ok):
        return False
    graph.replay()
    torch.cuda.synchronize(device)
    return agree(bool(torch.all(x == float(world)).item()))


def band_bounds(n: int, world: int, align: int = 128):
    """Row bands [(row0, row1)] of the packed upper triangle for `world`
    ranks: boundaries on multiples of `align` (the θ-grad's 128-row tiles),
    each band holding about 1/world of the triangle's entries (row i holds
    n − i of them), none empty."""
    if world < 1 or n < align * world:
        raise NotImplementedError(f"band-sharded exchange: n >= {align}·world (n = {n}, world = {world})")
    cum = lambda r: r * n - r * (r - 1) // 2  # noqa: E731  (entries of rows < r)
    total = cum(n)
    cuts = [0]
    for b in range(1, world):
        target = b * total / world
        r = min(range(cuts[-1] + align, n - align * (world - b) + 1, align), key=lambda x: abs(cum(x) - target))
        cuts.append(r)
    cuts.append(n)
    return [(cuts[b], cuts[b + 1]) for b in range(world)]


class BandShards:
    """The band-sharded exchange of the long-row engine (BASELINE config 5 at
    N > 1; LdsEngine.set_band_shards).  Rank b owns the packed
    triangle's rows [row0_b, row1_b): per hyper step it all-gathers every
    rank's θ-gradient factors (U, V, R: 2·n·K + n floats per rank, against
    the n(n+1)/2 floats of a dense dθ all-reduce), assembles, updates and
    clamps its own band of θ (lds_theta_grad_band), and at each window start
    draws its band's rows of EVERY replica's graphs (lds_sample_band_bits)
    and sends each replica's rows to its rank (all-to-all); the owner
    completes the lower triangle (lds_bitmask_mirror_degree).  Replica = rank
    (one sample per rank).  Under gloo the collectives run on host copies."""

    def __init__(self, n: int, world: Optional[int] = None, rank: Optional[int] = None, always: bool = False):
        """`always`: run the collectives at world size 1 too (the world-size-1
        RCCL rehearsal of tests/rccl_worker.py; a process group must be up)."""
        up = _group_up()
        self.world = int(world if world is not None else (dist.get_world_size() if up else 1))
        self.rank = int(rank if rank is not None else (dist.get_rank() if up else 0))
        if self.world > 1 and not up:
            raise RuntimeError("BandShards: a process group is needed for world > 1")
        self.n = n
        self.bounds = band_bounds(n, self.world)
        self.host = up and dist.get_backend() != "nccl"  # gloo: collectives on host copies
        self.always = bool(always) and up
        self._skip = self.world == 1 and not self.always  # world size 1: the collectives are identities

    @property
    def band(self):
        return self.bounds[self.rank]

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """[world, *t.shape], rank order."""
        if self._skip:
            return t.unsqueeze(0)
        src = t.contiguous().cpu() if self.host else t.contiguous()
        # (concatenated along dim 0, the form every backend accepts, then viewed)
        out = torch.empty((self.world * t.shape[0],) + tuple(t.shape[1:]), dtype=t.dtype, device=src.device)
        dist.all_gather_into_tensor(out, src)
        out = out.view((self.world,) + tuple(t.shape))
        return out.to(t.device) if self.host else out

    def all_to_all(self, send: torch.Tensor, send_splits, recv_splits) -> torch.Tensor:
        """all_to_all_single of a flat buffer: send_splits[q] elements to rank q,
        recv_splits[q] from rank q."""
        if self._skip:
            return send
        src = send.cpu() if self.host else send
        out = torch.empty(sum(recv_splits), dtype=send.dtype, device=src.device)
        dist.all_to_all_single(out, src, output_split_sizes=list(recv_splits), input_split_sizes=list(send_splits))
        return out.to(send.device) if self.host else out

    def exchange_rows(self, ab: torch.Tensor, dst: torch.Tensor) -> None:
        """The band all-to-all of the sharded draw: ab [count, world, n, W]
        holds (in this rank's band rows) every replica's graphs; dst
        [count, n, W] receives every band's rows of THIS rank's replica.  A
        band's rows travel from word row0 / 64 on — the bounding box of their
        upper-triangle words; the words below are lower triangle, which the
        owner's mirror writes — so each rank sends about 1/world of the
        triangle's bits (twice that for the last band, a triangle)."""
        count, W = ab.shape[0], ab.shape[3]
        if self._skip:
            dst.copy_(ab[:, 0])
            return
        row0, row1 = self.band
        box = [(q1 - q0) * (W - q0 // 64) for q0, q1 in self.bounds]
        send = ab[:, :, row0:row1, row0 // 64:].permute(1, 0, 2, 3).contiguous().view(-1)  # [dest, g, rows, box W]
        recv = self.all_to_all(send, [count * box[self.rank]] * self.world, [count * m for m in box])
        off = 0
        for q, (q0, q1) in enumerate(self.bounds):
            m = count * box[q]
            dst[:, q0:q1, q0 // 64:] = recv[off:off + m].view(count, q1 - q0, W - q0 // 64)
            off += m

    def gather_rows(self, flat: torch.Tensor, n: int) -> None:
        """Every rank's band of a packed triangle (θ) into every rank's copy,
        in place: after it all ranks hold the same full triangle."""
        if self._skip:
            return
        offs = [r0 * n - r0 * (r0 - 1) // 2 for r0, _ in self.bounds] + [flat.numel()]
        lens = [offs[b + 1] - offs[b] for b in range(self.world)]
        m = max(lens)
        mine = torch.zeros(m, dtype=flat.dtype, device=flat.device)
        b = self.rank
        mine[:lens[b]] = flat[offs[b]:offs[b + 1]]
        allv = self.all_gather(mine)
        for q in range(self.world):
            if q != b:
                flat[offs[q]:offs[q + 1]] = allv[q, :lens[q]]
