"""The round-3/4 forms of the dense-graph CSR-SpMM (the tools-only variants
library, tools/variants/libldsgnn_variants.so: row-block, column-pass and
every spill-pass configuration that led to the product)
still give the product's result bits (exact integer sums) on rows that take
every path: ragged n, dense and sparse rows, crowded first / last columns,
empty and full rows, several column passes.  They are no part of the product
library (test_native_abi.py::test_library_exports_only_declared_entry_points);
this test keeps the measured ablations reproducible."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools", "variants"))

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def variants():
    if not os.path.exists(os.path.join(ROOT, "tools", "variants", "libldsgnn_variants.so")):
        pytest.skip("tools/variants not built (make -C tools/variants)")
    import variants as v
    return v


def _csr(a):
    rows, cols = a.nonzero(as_tuple=True)
    rp = torch.zeros(a.size(0) + 1, dtype=torch.int64)
    rp[1:] = torch.cumsum(a.sum(1), 0)
    return rp, cols.int()


@pytest.mark.parametrize("n,shape,grid_codes", [(3001, "uniform", None), (6000, "shaped", None)])
def test_variants_equal_the_product(device, variants, n, shape, grid_codes):
    from ldsgnn import _native as nat
    g = torch.Generator().manual_seed(n)
    if shape == "uniform":
        a = torch.rand(n, n, generator=g) < 0.5
    else:
        dens = torch.rand(n, generator=g) * 0.6
        a = torch.rand(n, n, generator=g) < dens[:, None]
        a[0:40, 1000:] = False
        a[40:80, :4500] = False
        a[80:120] = torch.rand(40, n, generator=g) < 0.002
        a[120] = False
        a[121] = True
    rp, col = _csr(a)
    s = torch.rand(n, generator=g) + 0.5
    z = torch.randn(n, 16, generator=g)
    rpd, cold, sd, zd = rp.int().to(device), col.to(device), s.to(device), z.to(device)
    ws = torch.empty(variants.ws_bytes(n), dtype=torch.uint8, device=device)
    err = torch.zeros(1, dtype=torch.int32, device=device)
    y = torch.empty(n, 16, device=device)
    st = nat.stream_of(device)
    nat.call("lds_spmm_norm_dense", nat.ptr(rpd), nat.ptr(cold), nat.ptr(sd), n, nat.ptr(zd), 16, nat.ptr(y), 16, 0,
             nat.ptr(ws), 0, 1, nat.ptr(err), st)  # (leaves the digits of s, z in ws)
    torch.cuda.synchronize()
    assert int(err.item()) == 0
    for dbg in variants.SAME_RESULTS:
        yv = torch.empty(n, 16, device=device)
        variants.spmm_dense(nat.ptr(rpd), nat.ptr(cold), nat.ptr(sd), n, nat.ptr(zd), 16, nat.ptr(yv), 16,
                            nat.ptr(ws), dbg, st)
        torch.cuda.synchronize()
        assert torch.equal(yv.cpu(), y.cpu()), dbg


def test_product_buffer_clear_with_a_delayed_multiply_wave(device, variants):
    """Timing-independent check of the spill-pass kernel's buffer protocol
    (the race of round 4: buffers cleared by every multiply wave while a
    slower one still read them).  The PRODUCT kernel (csrc/spill.hpp), built
    with multiply wave 12 sleeping after every pass barrier, so that it is the
    last to finish each buffer, must give the undelayed product's exact sums.
    n = 16384 on 171 workgroups (96 rows each) is 4 column passes, so every
    pass buffer is cleared and filled again (pass 3 reuses pass 0's)."""
    from ldsgnn import _native as nat
    n, grid = 16384, 171
    g = torch.Generator(device=device).manual_seed(7)
    dens = torch.rand(n, generator=g, device=device) * 0.08
    a = torch.rand(n, n, generator=g, device=device) < dens[:, None]
    rows, cols = a.nonzero(as_tuple=True)
    rp = torch.zeros(n + 1, dtype=torch.int32, device=device)
    rp[1:] = torch.cumsum(a.sum(1), 0).int()
    col = torch.empty(((cols.numel() + 3) // 4) * 4, dtype=torch.int32, device=device)
    col[:cols.numel()] = cols.int()
    del a, rows, cols
    s = torch.rand(n, generator=g, device=device) + 0.5
    z = torch.randn(n, 16, generator=g, device=device)
    ws = torch.empty(variants.ws_bytes(n), dtype=torch.uint8, device=device)
    err = torch.zeros(1, dtype=torch.int32, device=device)
    st = nat.stream_of(device)
    y = torch.empty(n, 16, device=device)
    nat.call("lds_spmm_norm_dense", nat.ptr(rp), nat.ptr(col), nat.ptr(s), n, nat.ptr(z), 16, nat.ptr(y), 16, 0,
             nat.ptr(ws), grid, 1, nat.ptr(err), st)  # (leaves the digits of s, z in ws)
    y_tile = torch.empty(n, 16, device=device)
    nat.call("lds_spmm_norm_dense", nat.ptr(rp), nat.ptr(col), nat.ptr(s), n, nat.ptr(z), 16, nat.ptr(y_tile), 16,
             0, nat.ptr(ws), -256, 0, 0, st)  # the tile kernel: any order, no pass buffers
    torch.cuda.synchronize()
    assert int(err.item()) == 0
    assert torch.equal(y, y_tile)
    for delay in (1, 4):
        yd = torch.full((n, 16), float("nan"), device=device)
        variants.spmm_dense_delayed(nat.ptr(rp), nat.ptr(col), nat.ptr(s), n, nat.ptr(yd), 16, nat.ptr(ws), grid,
                                    delay, nat.ptr(err), st)
        torch.cuda.synchronize()
        assert int(err.item()) == 0
        assert torch.equal(yd, y), delay
