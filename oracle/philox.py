"""TEST INFRASTRUCTURE — CPU oracle, never shipped, never on the product path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
anything under oracle/.

Philox4x32-10 (Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as easy as
1, 2, 3", SC'11 — the generator the Random123 library publishes) restated with
vectorised numpy uint64 arithmetic, plus the uniform map the product uses
(include/ldsgnn.h, "RNG contract"):

    key = (seed & 0xffffffff, seed >> 32)
    ctr = (column, row >> 2, tag, counter)
    u(row, column) = (out[row & 3] >> 8) * 2**-24

The reference draws its randomness from torch's mt19937 stream
(`Bernoulli(probs).sample()`, src/models/sampling.py:68; `F.dropout`,
src/models/gcn.py:27,29).  The product instead keys every draw, so that the GPU
and this oracle produce identical edge sets and dropout masks; parity with the
reference's own stream is shown separately by injecting torch.rand uniforms
(tests/golden, "injected-U" mode).
"""
from __future__ import annotations

import numpy as np

_M0 = np.uint64(0xD2511F53)
_M1 = np.uint64(0xCD9E8D57)
_W0 = 0x9E3779B9
_W1 = 0xBB67AE85
_MASK = np.uint64(0xFFFFFFFF)
_S32 = np.uint64(32)

# Tags (include/ldsgnn.h): consumer in the top byte, replica in the low 24 bits.
TAG_GRAPH = 1 << 24
TAG_DROP_X = 2 << 24
TAG_DROP_H = 3 << 24


def tag_for(kind: int, replica: int = 0) -> int:
    return (kind | (replica & 0xFFFFFF)) & 0xFFFFFFFF


def philox4x32_10(c0, c1, c2, c3, k0: int, k1: int):
    """Vectorised Philox4x32-10; counters are broadcastable integer arrays."""
    c0 = np.asarray(c0, dtype=np.uint64) & _MASK
    c1 = np.asarray(c1, dtype=np.uint64) & _MASK
    c2 = np.asarray(c2, dtype=np.uint64) & _MASK
    c3 = np.asarray(c3, dtype=np.uint64) & _MASK
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    k0 = int(k0) & 0xFFFFFFFF
    k1 = int(k1) & 0xFFFFFFFF
    for _ in range(10):
        p0 = _M0 * c0
        p1 = _M1 * c2
        hi0, lo0 = p0 >> _S32, p0 & _MASK
        hi1, lo1 = p1 >> _S32, p1 & _MASK
        c0, c1, c2, c3 = (hi1 ^ c1 ^ np.uint64(k0)), lo1, (hi0 ^ c3 ^ np.uint64(k1)), lo0
        k0 = (k0 + _W0) & 0xFFFFFFFF
        k1 = (k1 + _W1) & 0xFFFFFFFF
    return c0, c1, c2, c3


def uniform(seed: int, tag: int, counter: int, rows: int, cols: int) -> np.ndarray:
    """u(i, j) for a rows×cols block, float32, as lds_philox_uniform writes it."""
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    k0, k1 = seed & 0xFFFFFFFF, seed >> 32
    quads = (rows + 3) // 4
    j = np.arange(cols, dtype=np.uint64)[None, :]
    q = np.arange(quads, dtype=np.uint64)[:, None]
    o = philox4x32_10(j, q, np.uint64(tag), np.uint64(counter), k0, k1)
    out = np.empty((quads, 4, cols), dtype=np.float32)
    for r in range(4):
        out[:, r, :] = (o[r] >> np.uint64(8)).astype(np.float32) * np.float32(2.0 ** -24)
    return out.reshape(quads * 4, cols)[:rows]


def uniform_rows(seed: int, tag: int, counter: int, row_ids: np.ndarray, cols: int) -> np.ndarray:
    """u(i, j) for selected rows only (len(row_ids)×cols) — cheap for large N."""
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    k0, k1 = seed & 0xFFFFFFFF, seed >> 32
    row_ids = np.asarray(row_ids, dtype=np.int64)
    j = np.arange(cols, dtype=np.uint64)[None, :]
    q = (row_ids >> 2).astype(np.uint64)[:, None]
    o = np.stack(philox4x32_10(j, q, np.uint64(tag), np.uint64(counter), k0, k1))  # 4×R×C
    sel = o[row_ids & 3, np.arange(len(row_ids))]
    return (sel >> np.uint64(8)).astype(np.float32) * np.float32(2.0 ** -24)
