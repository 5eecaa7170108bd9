"""ctypes binding of the C-ABI hot-path library (include/ldsgnn.h).

The library is built in-tree (lds-gnn_amd/csrc/Makefile -> ldsgnn/libldsgnn.so)
and loaded AFTER torch so that it binds to the HIP runtime torch already
loaded (same SONAME libamdhip64.so.7): our kernels then run on torch's
streams and inside torch's HIP graphs.  There is no fallback: if the library
is missing, importing ldsgnn raises.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL: shared HIP runtime)

LIB_PATH = os.environ.get("LDSGNN_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libldsgnn.so")
ABI_VERSION = 18

c_int, c_int64, c_uint32, c_uint64, c_float, c_void_p = (
    ctypes.c_int, ctypes.c_int64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_float, ctypes.c_void_p)
P = c_void_p  # device pointers travel as integers

# name -> argtypes (restype is always int = hipError_t, except where noted)
_RESTYPE_I64 = {"lds_bitmask_agg_ws_bytes", "lds_bitmask_agg_part_offset", "lds_planes_t128_elems", "lds_spmm_dense_ws_bytes"}  # byte counts
SIGNATURES = {
    "lds_abi_version": [],
    "lds_graph_node_census": [P, P, c_int],
    "lds_graph_upload": [P, P],
    "lds_bitmask_words": [c_int],
    "lds_philox_uniform": [c_uint64, c_uint32, c_uint32, c_int, c_int, P, P],
    "lds_sample_bitmask": [P, c_int, c_uint64, c_uint32, c_uint32, P, P, c_int, P],
    "lds_bitmask_degree": [P, c_int, c_int, P, P, P],
    "lds_exclusive_scan": [P, c_int, P, P],
    "lds_bitmask_fill_csr": [P, c_int, c_int, P, P, c_int64, P, P],
    "lds_csr_degree_scale": [P, c_int, P, P, P],
    "lds_sample_graphs": [P, c_int, c_uint64, c_uint32, P, c_uint32, c_int, P, c_int, P, P, P, c_int64, P, P,
                          P],
    "lds_sample_graphs_multi": [P, c_int, c_uint64, c_uint32, c_uint32, P, c_uint32, c_int, c_int, P, c_int, P,
                                P, P, c_int64, P, P, P, c_int, P, P],
    "lds_sample_ws_ints": [c_int],
    "lds_sample_fill_csr": [P, c_int, c_int, P, c_int, P, P, c_int64, P, P, P, P, P],
    "lds_sgd_sample_graphs": [P, P, P, c_int, c_uint64, c_uint32, c_uint32, c_uint32, c_int, c_int, P, c_int, P,
                              P, P],
    "lds_sgd_tile_ints": [c_int],
    "lds_sample_band_bits": [P, c_int, c_uint64, c_uint32, c_uint32, P, c_uint32, c_int, c_int, c_int, c_int, P,
                             c_int, P],
    "lds_bitmask_mirror_degree": [P, c_int, c_int, c_int, P, P, P],
    "lds_theta_grad_band": [P, P, c_int, c_int, P, c_int, c_int, c_int, P, c_int, P, c_int, P, c_float, c_int,
                            c_int, P],
    "lds_theta_grad_ex": [P, P, c_int, c_int, P, c_int, c_int, c_int, P, c_int, P, c_int, P, c_float, c_int, P],
    "lds_theta_grad_planes": [P, P, c_int, c_int, P, c_int, c_int, c_int, P, c_int, P, c_int, P, c_float, c_int,
                              P],
    "lds_split_planes": [P, c_int, c_int, c_int, P, P],
    "lds_planes_t128_elems": [c_int, c_int],
    "lds_split_planes_t128": [P, c_int, c_int, c_int, P, P],
    "lds_theta_grad_direct": [P, P, c_int, P, c_int, c_int, c_int, P, c_int, P, c_int, P, c_float, c_uint64, c_uint32,
                              P, c_uint32, c_int, P, c_int, P, P],
    "lds_bitmask_fill_csr_ell": [P, c_int, c_int, P, P, c_int64, P, P, P, P],
    "lds_sample_graph": [P, c_int, c_uint64, c_uint32, c_uint32, P, P, c_int, P, P, P, c_int64, P,
                         P, P],
    "lds_spmm_norm": [P, P, P, c_int, P, c_int, c_int, P, c_int, c_int, P],
    "lds_spmm_block_count": [c_int],
    "lds_csr_block_ptr": [P, P, c_int, P, P],
    "lds_spmm_norm_blocked": [P, P, P, c_int, P, c_int, P, c_int, c_int, P, P],
    "lds_bitmask_agg_ws_bytes": [c_int],
    "lds_aggregate_bitmask": [P, c_int, P, c_int, P, c_int, P, c_int, c_int, P, P],
    "lds_bitmask_agg_splits": [c_int],
    "lds_bitmask_agg_part_offset": [c_int],
    "lds_aggregate_bitmask_partials": [P, c_int, P, c_int, P, c_int, P, P],
    "lds_spmm_dense_ws_bytes": [c_int],
    "lds_spmm_dense_max_n": [],
    "lds_spmm_norm_dense": [P, P, P, c_int, P, c_int, P, c_int, c_int, P, c_int, c_int, P, P],
    "lds_theta_grad": [P, P, c_int, c_int, P, c_int, c_int, P, c_int, P, c_int, c_int, P],
    "lds_theta_grad_valu": [P, P, c_int, c_int, P, c_int, c_int, P, c_int, P, c_int, P],
    "lds_theta_grad_sgd": [P, P, c_int, c_int, P, c_int, c_int, P, c_int, P, P, c_int, P],
    "lds_theta_grad_sgd_accum": [P, P, c_int, c_int, P, c_int, c_int, P, c_int, P, P, c_int, P],
    "lds_theta_grad_sgd_draw": [P, P, c_int, c_int, P, c_int, c_int, P, c_int, P, P, c_uint64, c_uint32, P,
                                c_uint32, c_int, P, c_int, P, c_int, P],
    "lds_slot_factors": [P, c_int, P, c_int, P, c_int, P, c_int, P, c_int, c_int, c_int, P, c_int, P,
                         c_int, P, c_int, P],
    "lds_sgd_clamp": [P, P, c_float, c_int64, P],
    "lds_pretrain_step": [P, c_int, P, c_int, c_float, P, P, c_int, ctypes.c_double, ctypes.c_double,
                          ctypes.c_double, ctypes.c_double, P, P],
    "lds_dropout": [P, c_int, P, c_int, c_int, c_int, c_float, c_float, c_uint64, c_uint32, c_uint32,
                    P],
    # fused engine (csrc/engine.hip)
    "lds_engine_scalars_size": [],
    "lds_sample_bitmask_dev": [P, c_int, c_uint64, c_uint32, P, c_uint32, P, c_int, P],
    "lds_engine_x_linear": [P, P, P, c_int, P, P, P, c_uint64, c_uint32, P, c_int, c_int, c_float, c_float,
                            P, P, P, P, P, c_int, P, P],
    "lds_engine_fill_x_linear": [P, c_int, P, c_int, P, P, c_int64, P, P, P,
                                 P, P, P, c_int, P, P, P, c_uint64, c_uint32, P, c_int, c_int, c_float, c_float,
                                 P, P, P, P, P, c_int, P, P],
    "lds_engine_xt_linear": [P, P, P, c_int, P, P, P, c_float, c_int, c_uint64, c_uint32, P, c_int, c_int,
                             c_float, c_float, P],
    "lds_engine_fwd_layer1": [P, P, P, P, c_int, P, P, P, P, P, P, c_int, c_uint64, c_uint32, P, c_int, c_int,
                              c_float, c_float, P, P, P, P],
    "lds_engine_fwd_layer2": [P, P, P, P, c_int, P, P, P, P, P, P, c_float, P, P, c_int, P, P, P],
    "lds_engine_bwd_layer2": [P, P, P, P, c_int, P, P, P, P, P, c_int, c_uint64, c_uint32, P, c_int, c_int,
                              c_float, c_float, P, P, P, P, c_int, P, c_int, c_int, c_int, P, P, P, P],
    "lds_engine_bwd_layer1": [P, P, P, P, c_int, P, P, P, P, P, P, c_int, P, c_int, P],
    "lds_engine_colreduce": [c_int, c_int, P, P, P, P, P, P, P, P, P, c_int, P, P, c_int, P, c_int, P, c_int,
                             P],
    "lds_engine_adam": [c_int, P, P, P, P, P, P, P, P, P, P, c_int, P, c_int, P],
    "lds_engine_adam_reverse": [c_int, P, P, P, P, P, P, P, P, P, c_int, P, c_int, P],
    "lds_engine_rev_a": [P, P, P, P, c_int, P, P, P, P, P, P, P, P, P, c_int, P, P, P, c_uint64, c_uint32, P,
                         c_int, c_int, c_float, c_float, P, P, c_int, P, c_int, P, P, P, P],
    "lds_engine_rev_b": [P, P, P, P, c_int, P, P, P, P, P, c_float, c_int, P, P, P, c_int, P, c_int, c_int, P, P, P],
    "lds_engine_rev_c": [P, P, P, P, c_int, P, P, P, P, P, P, c_int, P, P, c_uint64, c_uint32, P, c_int, c_int,
                         c_float, c_float, P, P, c_int, P, c_int, c_int, P, P, P, P],
    "lds_engine_rev_d": [P, P, P, P, c_int, P, P, P, P, P, P, c_int, P, c_int, P],
    "lds_engine_sgd_clamp": [P, P, c_int64, P, P],
    "lds_engine_advance": [P, c_int, c_int, c_int, c_int, P],
    # fused forms
    "lds_engine_bwd1_reduce": [P, P, P, P, c_int, P, P, P, P, P, P, c_int, P, c_int, P, P, P, P, c_int, P, P, P, P],
    "lds_engine_rev_d_reduce": [P, P, P, P, c_int, P, P, P, P, P, P, c_int, P, c_int, P, P, P, P, c_int, P, P, P, P],
    "lds_engine_final": [P, c_int, c_int, P, c_int, c_int, c_int, c_int, P, c_int, c_int, P, P, P, P, P, P, P,
                         P, P, P, P, P, P, c_int, P, c_int, P],
    "lds_engine_xt_adam": [P, P, P, c_int, P, P, c_int, c_uint64, c_uint32, P, c_int, c_int, c_float, c_float,
                           P, c_int, c_int, c_int, c_int, c_int, P,
                           c_int, c_int, P, P, P, P, P, P, P, P, P, P, P, P, P, c_int, c_int, P, c_int, P, c_int, P, P,
                           c_int, c_int, P, P],
    "lds_engine_xt_partials": [P, P, P, c_int, P, c_uint64, c_uint32, P, c_int, c_int, c_float, c_float, c_int, P,
                               P, P],
    "lds_engine_fwd2_bwd2": [P, P, P, P, c_int, P, c_int, P, P, P, P, P, c_float, P, P, c_int, P, P, P, P,
                             c_uint64, c_uint32, P, c_int, c_int, c_float, c_float, P, P, c_int, P, c_int, c_int,
                             c_int, P, P, P],
    "lds_engine_rev_bc": [P, P, P, P, c_int, P, c_int, P, P, P, P, P, P, c_float, c_int, P, P, P, P, P, c_uint64,
                          c_uint32, P, c_int, c_int, c_float, c_float, P, P, c_int, P, c_int, c_int, c_int, P, P, P],
    "lds_engine_end_window": [c_int, P, P, P, P, P, P, P, c_int, c_int, c_int, c_int, P, P, c_int, P, P, c_int64,
                              P, P],
    "lds_engine_adam_table": [P, P, P, c_int, P],
}


class NativeError(RuntimeError):
    """A hot-path entry point returned a HIP error."""


class DeviceError(RuntimeError):
    """A kernel reported an input it could not use faithfully through a
    device error word (include/ldsgnn.h "Device error word")."""


DEVERR_FILL_DEGREE = 1  # LDS_DEVERR_FILL_DEGREE
DEVERR_CSR_COLUMNS = 2  # LDS_DEVERR_CSR_COLUMNS (ABI 14)
DEVERR_SGD_TILE_COUNTER = 4  # LDS_DEVERR_SGD_TILE_COUNTER (round 6)

_DEVERR_TEXT = {DEVERR_FILL_DEGREE: "a CSR fill found a row whose degree count differs from its drawn bits "
                                    "(degree workspace not zero on entry, or counts of another draw); its "
                                    "slots past the drawn entries hold the row's own index",
                DEVERR_CSR_COLUMNS: "the dense CSR-SpMM (lds_spmm_norm_dense) met a row whose columns are not "
                                    "ascending in a way that changes its sum, or a column outside [0, n): the "
                                    "aggregation is wrong",
                DEVERR_SGD_TILE_COUNTER: "the SGD + draw pass (lds_sgd_sample_graphs) found a per-tile counter "
                                         "that was not zero on entry: θ and the draws of that pass are not "
                                         "trustworthy"}


def raise_device_error(word: int, what: str) -> None:
    """Raise DeviceError for a non-zero device error word."""
    if word:
        msgs = [t for b, t in _DEVERR_TEXT.items() if word & b] or [f"unknown bits {word:#x}"]
        raise DeviceError(f"{what}: device error word {word:#x}: " + "; ".join(msgs))


def _load() -> ctypes.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"ldsgnn native library not found at {LIB_PATH}: build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (make -C lds-gnn_amd/csrc). "
            "There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    for name, argtypes in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = ctypes.c_int64 if name in _RESTYPE_I64 else c_int
    lib.lds_error_string.argtypes = [c_int]
    lib.lds_error_string.restype = ctypes.c_char_p
    v = lib.lds_abi_version()
    if v != ABI_VERSION:
        raise ImportError(f"libldsgnn ABI {v} != expected {ABI_VERSION}; rebuild")
    return lib


lib = _load()


def check(err: int, what: str = "") -> None:
    if err != 0:
        msg = lib.lds_error_string(err).decode(errors="replace")
        raise NativeError(f"{what or 'ldsgnn'} failed: hip error {err} ({msg})")


class KernelTimer:
    """Optional HIP-event timing of selected entry points on the current
    stream (bench.py's roofline leg): start/end events around each launch."""

    def __init__(self):
        self.names = set()
        self.events = {}
        self.all = False

    def enable(self, *names):
        self.names = set(names)
        self.events = {n: [] for n in names}
        self.all = False

    def enable_all(self):
        """Time every entry point (bench.py's per-window breakdown)."""
        self.names = set(SIGNATURES)
        self.events = {}
        self.all = True

    def disable(self):
        self.names = set()
        self.all = False

    def summary(self):
        torch.cuda.synchronize()
        out = {}
        for n, evs in self.events.items():
            ms = [a.elapsed_time(b) for a, b in evs]
            out[n] = dict(launches=len(ms), total_ms=float(sum(ms)),
                          avg_us=float(1000.0 * sum(ms) / len(ms)) if ms else 0.0)
        return out


timer = KernelTimer()


def call(name: str, *args) -> None:
    if name not in SIGNATURES:  # an untyped ctypes call would truncate pointers to int
        raise KeyError(f"{name} has no ctypes signature in ldsgnn._native.SIGNATURES")
    if name in timer.names:
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        err = getattr(lib, name)(*args)
        b.record()
        timer.events.setdefault(name, []).append((a, b))
        check(err, name)
        return
    check(getattr(lib, name)(*args), name)


# hipGraphNodeType values a captured step or window may hold: kernel launches
# and the empty nodes a capture inserts where streams join
_GRAPH_NODE_OK = {0: "kernel", 5: "empty"}
_GRAPH_NODE_NAMES = {1: "memcpy", 2: "memset", 3: "host", 4: "child graph", 6: "event wait", 7: "event record",
                     10: "mem alloc", 11: "mem free", 12: "memcpy from symbol", 13: "memcpy to symbol"}


def new_graph() -> "torch.cuda.CUDAGraph":
    """A HIP graph whose capture is inspected before instantiation
    (seal_graph)."""
    return torch.cuda.CUDAGraph(keep_graph=True)


# seal_graph uploads every instantiated capture (hipGraphUpload) before its
# first replay
UPLOAD_GRAPHS = True


# ... and, in a window that captures the replicas' exchange (an RCCL
# collective), the event nodes a collective library may add to order its own
# stream against the capture
_GRAPH_NODE_OK_EXCHANGE = {**_GRAPH_NODE_OK, 6: "event wait", 7: "event record"}


def graph_census(graph: "torch.cuda.CUDAGraph") -> dict:
    """{node type name: count} of a captured (not yet instantiated) graph."""
    counts = (ctypes.c_int * 16)()
    call("lds_graph_node_census", graph.raw_cuda_graph(), ctypes.addressof(counts), 16)
    names = {**_GRAPH_NODE_NAMES, **_GRAPH_NODE_OK}
    return {names.get(t, f"type {t}"): c for t, c in enumerate(counts) if c}


def seal_graph(graph: "torch.cuda.CUDAGraph", what: str, exchange: bool = False) -> "torch.cuda.CUDAGraph":
    """Refuse a captured graph that holds anything but kernel (and empty)
    nodes, then instantiate it.  A memset node in a replayed step graph
    faulted the GPU in round 2; every clear the engine needs is a
    kernel, and this keeps any other node type from entering a capture: the
    failure is a host-side error at capture time, never a GPU fault.
    `exchange`: the capture holds the replicas' collective, whose event
    nodes are allowed too (never a memset or memcpy)."""
    counts = (ctypes.c_int * 16)()
    call("lds_graph_node_census", graph.raw_cuda_graph(), ctypes.addressof(counts), 16)
    ok = _GRAPH_NODE_OK_EXCHANGE if exchange else _GRAPH_NODE_OK
    bad = {_GRAPH_NODE_NAMES.get(t, f"type {t}"): c for t, c in enumerate(counts) if c and t not in ok}
    if bad:
        raise RuntimeError(f"captured {what} holds non-kernel graph nodes {bad}: refusing to replay it")
    graph.instantiate()
    if UPLOAD_GRAPHS:  # the executable uploaded now, not on its first replay
        call("lds_graph_upload", graph.raw_cuda_graph_exec(), stream_of(torch.cuda.current_device()))
    return graph


class LdsBatch(ctypes.Structure):
    """include/ldsgnn.h LdsBatch: per-sample element strides of a batched
    engine launch (S replica samples in one launch, grid.y = sample)."""
    _fields_ = [("samples", ctypes.c_int32), ("tag_step", ctypes.c_uint32)] + [
        (f, ctypes.c_int64) for f in ("act", "row", "rp", "col", "ell", "par", "xval", "xd", "uv", "part", "met")] + [
        ("heavy_rows", ctypes.c_void_p), ("heavy_flag", ctypes.c_void_p), ("n_heavy", ctypes.c_int32),
        ("agg_splits", ctypes.c_int32), ("xt_pair", ctypes.c_int32)]


def batch_ptr(b) -> int:
    """Address of an LdsBatch (None -> NULL = one sample)."""
    return 0 if b is None else ctypes.addressof(b)


def ptr(t) -> int:
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return 0
    return t.data_ptr()


def stream_of(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_device(t: torch.Tensor, what: str) -> None:
    if not t.is_cuda:
        raise RuntimeError(
            f"ldsgnn {what}: tensors must live on a HIP device (got {t.device}); "
            "the hot path has no CPU implementation")
