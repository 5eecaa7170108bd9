"""ctypes loader of the tools-only variants library (tools/variants/
libldsgnn_variants.so, built by `make -C tools/variants` and by
__graft_entry__.build()): the non-product forms of the dense-graph CSR-SpMM
that rounds 3-4 measured.  Loaded by the ablation tools and
tests/test_spmm_variants_gpu.py only; nothing in the product imports it."""
import ctypes
import os

import torch  # noqa: F401  (before the CDLL: the shared HIP runtime)

from ldsgnn import _native as nat

PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libldsgnn_variants.so")
P, c_int = ctypes.c_void_p, ctypes.c_int
_lib = None

# codes whose results equal the product's (exact integer sums); the others are
# timing-only ablations
SAME_RESULTS = (6, 20, 21, 22, 23, 33, 34, 35, 36, 37, 38, 39, 41, 42, 43, 44, 45, 46, 47, 48, 49, 50, 51, 52, 53,
                54, 55, 56, 57, 60, 61, 62, 63, 64, 65, 66, 67, 68, 69)
ANY_ORDER = (6, 22)  # the row-block kernel accepts columns in any order


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(PATH):
            raise ImportError(f"{PATH} missing: make -C tools/variants")
        _lib = ctypes.CDLL(PATH)
        _lib.lds_variants_ws_bytes.argtypes = [c_int]
        _lib.lds_variants_ws_bytes.restype = ctypes.c_int64
        _lib.lds_variants_spmm_dense.argtypes = [P, P, P, c_int, P, c_int, P, c_int, P, c_int, P]
        _lib.lds_variants_spmm_dense.restype = c_int
        _lib.lds_variants_spmm_dense_delayed.argtypes = [P, P, P, c_int, P, c_int, P, c_int, c_int, P, P]
        _lib.lds_variants_spmm_dense_delayed.restype = c_int
        _lib.lds_variants_spmm_dense_nt.argtypes = [P, P, P, c_int, P, c_int, P, c_int, P, P]
        _lib.lds_variants_spmm_dense_nt.restype = c_int
    return _lib


def ws_bytes(n: int) -> int:
    """Workspace for both the product (lds_spmm_norm_dense) and the variants."""
    return max(int(lib().lds_variants_ws_bytes(n)), int(nat.lib.lds_spmm_dense_ws_bytes(n)))


def spmm_dense(rp, col, s, n, z, ldz, y, ldy, ws, dbg, stream):
    """Variant `dbg` (pointers as ints); the digits of s, z must be in ws from
    an lds_spmm_norm_dense call on the same workspace."""
    nat.check(lib().lds_variants_spmm_dense(rp, col, s, n, z, ldz, y, ldy, ws, dbg, stream),
              f"lds_variants_spmm_dense({dbg})")


def spmm_dense_delayed(rp, col, s, n, y, ldy, ws, grid, delay, err, stream):
    """The product spill-pass kernel with multiply wave 12 delayed after every
    pass barrier (delay 1 or 4): the timing-independent buffer-clear check."""
    nat.check(lib().lds_variants_spmm_dense_delayed(rp, col, s, n, y, ldy, ws, grid, delay, err, stream),
              f"lds_variants_spmm_dense_delayed({delay})")


def spmm_dense_nt(rp, col, s, n, y, ldy, ws, grid, err, stream):
    """The product spill-pass kernel with its column stream loaded with the
    non-temporal policy; the digits must be in ws (as spmm_dense)."""
    nat.check(lib().lds_variants_spmm_dense_nt(rp, col, s, n, y, ldy, ws, grid, err, stream),
              "lds_variants_spmm_dense_nt")
