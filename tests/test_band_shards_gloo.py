"""The band-sharded exchange's host logic on the CPU (ldsgnn.replicas
band_bounds / BandShards; BASELINE config 5 at N > 1): the row
bands tile the triangle on 128-row boundaries with balanced entry counts, and
the three collectives the engine uses (factor all-gather, band all-to-all,
θ row gather) move exactly the right rows, over gloo with world size 2 and 3."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ldsgnn.replicas import BandShards, band_bounds


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("n,world", [(20000, 8), (1100, 2), (2708, 4), (2708, 3), (256, 2)])
def test_band_bounds_cover_the_triangle(n, world):
    b = band_bounds(n, world)
    assert b[0][0] == 0 and b[-1][1] == n and len(b) == world
    cum = lambda r: r * n - r * (r - 1) // 2  # noqa: E731
    sizes = []
    for (r0, r1), nxt in zip(b, b[1:] + [(n, n)]):
        assert r0 < r1 and r0 % 128 == 0 and r1 == nxt[0]
        sizes.append(cum(r1) - cum(r0))
    if n >= 2048 * world:  # fine enough rows: balanced within 10 %
        assert max(sizes) <= 1.1 * sum(sizes) / world, sizes


def test_band_bounds_refuse_too_few_rows():
    with pytest.raises(NotImplementedError):
        band_bounds(300, 4)


def _worker(rank, world, port, n, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sh = BandShards(n)
    assert sh.world == world and sh.rank == rank and sh.host
    # factor all-gather: rank order
    u = torch.full((n, 3), float(rank))
    g = sh.all_gather(u)
    assert g.shape == (world, n, 3) and all(float(g[q, 0, 0]) == q for q in range(world))
    # band rows of every replica's graphs to their owners (the engine's pack / unpack)
    count, W = 2, (n + 63) // 64 + 1
    ab = torch.zeros((count, world, n, W), dtype=torch.int64)
    r0, r1 = sh.band
    for q in range(world):  # my band's rows of replica q's graphs: tagged (writer, replica, row)
        rows = torch.arange(r0, r1, dtype=torch.int64)
        ab[:, q, r0:r1, :] = (rank * 1000000 + q * 100000 + rows)[None, :, None]
    dst = torch.full((count, n, W), -7, dtype=torch.int64)
    sh.exchange_rows(ab, dst)
    want = torch.full_like(dst, -7)
    for q, (q0, q1) in enumerate(sh.bounds):  # row i came from the rank owning it, for MY replica,
        rws = torch.arange(q0, q1, dtype=torch.int64)  # from word q0 / 64 on (the band's box)
        want[:, q0:q1, q0 // 64:] = (q * 1000000 + rank * 100000 + rws)[None, :, None]
    assert torch.equal(dst, want)
    # θ row gather: each rank's band into everyone's copy
    m = n * (n + 1) // 2
    theta = torch.full((m,), -1.0)
    off0 = r0 * n - r0 * (r0 - 1) // 2
    off1 = r1 * n - r1 * (r1 - 1) // 2
    theta[off0:off1] = float(rank)
    sh.gather_rows(theta, n)
    out[rank] = theta
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_band_shards_collectives(world):
    n = 128 * world + 70
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), n, out), nprocs=world, join=True)
    b = band_bounds(n, world)
    for r in range(world):
        th = out[r]
        for q, (r0, r1) in enumerate(b):
            o0, o1 = r0 * n - r0 * (r0 - 1) // 2, r1 * n - r1 * (r1 - 1) // 2
            assert bool((th[o0:o1] == q).all()), (r, q)
        assert torch.equal(th, out[0])
