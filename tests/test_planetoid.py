"""Planetoid fixtures (tests/golden/planetoid_*.npz, made by
tools/make_planetoid_fixtures.py with the data-only pickle reader) against the
facts the reference's own tests pin, and the reader's refusal to execute.

Pins: Cora 2708 nodes / 1433 features / 7 classes / 10 556 directed edges
(SURVEY §4); largest connected component 2485 nodes
(tst/data/test_data.py:128-132) holding 5069 undirected edges
(tst/data/test_transforms.py:69-72); Citeseer LCC 2120 nodes (the value the
reference's torch_geometric reader gives, tst/data/test_data.py:135-139 TODO);
Planetoid split sizes 140 / 120 train, 500 val, 1000 test."""
import os

import numpy as np
import pytest
import torch
from scipy.sparse import coo_matrix
from scipy.sparse.csgraph import connected_components

from ldsgnn.data.planetoid import FIXTURE_DIR, load_planetoid_npz, materialize, read_pickle_data


def _lcc(adj: torch.Tensor):
    a = coo_matrix(adj.numpy())
    _, lab = connected_components(a, directed=False)
    big = np.bincount(lab).argmax()
    keep = lab == big
    sub = adj.numpy()[np.ix_(keep, keep)]
    return int(keep.sum()), int(sub.sum())


def test_cora_fixture_pins():
    d = load_planetoid_npz("cora")
    assert tuple(d.x.shape) == (2708, 1433) and d.num_classes == 7
    assert int(d.dense_adj.sum()) == 10556
    assert torch.equal(d.dense_adj, d.dense_adj.t()) and float(d.dense_adj.diagonal().abs().sum()) == 0.0
    assert (int(d.train_mask.sum()), int(d.val_mask.sum()), int(d.test_mask.sum())) == (140, 500, 1000)
    assert not bool((d.train_mask & d.val_mask).any() | (d.val_mask & d.test_mask).any())
    nodes, entries = _lcc(d.dense_adj)
    assert nodes == 2485 and entries == 5069 * 2
    # NormalizeFeatures: rows sum to 1 (Cora has no empty feature rows)
    assert torch.allclose(d.x.sum(1), torch.ones(2708))


def test_citeseer_fixture_pins():
    d = load_planetoid_npz("citeseer")
    assert tuple(d.x.shape) == (3327, 3703) and d.num_classes == 6
    assert int(d.dense_adj.sum()) == 9104
    assert (int(d.train_mask.sum()), int(d.val_mask.sum()), int(d.test_mask.sum())) == (120, 500, 1000)
    nodes, _ = _lcc(d.dense_adj)
    assert nodes == 2120


@pytest.mark.skipif(not os.path.isdir("/root/reference/tst/res"), reason="reference resources absent")
def test_reader_reproduces_fixture():
    from ldsgnn.data.planetoid import read_planetoid_raw
    for name in ("cora", "citeseer"):
        d = read_planetoid_raw(f"/root/reference/tst/res/{name}/raw", name)
        z = np.load(os.path.join(FIXTURE_DIR, f"planetoid_{name}.npz"))
        assert np.array_equal(d["y"], z["y"]) and np.array_equal(d["edge_index"], z["edge_index"])
        assert np.array_equal(d["x"] != 0, np.asarray(load_planetoid_npz(name, normalize_features=False).x) != 0)


def test_reader_executes_nothing():
    """A pickle that would run os.system under pickle.loads stays an inert
    symbol here, and rebuilding it is refused."""
    payload = b"cos\nsystem\n(S'echo pwned'\ntR."
    node = read_pickle_data(payload)
    assert type(node).__name__ == "_Call" and node.fn.qual == "os.system"
    with pytest.raises(ValueError):
        materialize(node)
    with pytest.raises(ValueError):  # opcodes outside the data subset
        read_pickle_data(b"\x80\x04\x95\x05\x00\x00\x00\x00\x00\x00\x00\x8c\x01a\x94.".replace(b"\x8c\x01a\x94", b"\x93"))


def test_pretrain_split_and_bitmask():
    """GAE.split_edges restatement: 5 % / 10 % positives, equal negatives,
    disjoint, negatives are non-edges; the training adjacency's bitmask uses
    the sampler's layout (bit j%64 of word j/64)."""
    from ldsgnn.trainers.pretrainer import edges_to_bits, split_edges
    d = load_planetoid_npz("cora")
    sp = split_edges(d.dense_adj, generator=torch.Generator().manual_seed(0))
    e = 5278
    assert sp["val_pos"].shape[1] == e * 5 // 100 and sp["test_pos"].shape[1] == e * 10 // 100
    assert sp["train_pos"].shape[1] == 2 * (e - e * 5 // 100 - e * 10 // 100)
    assert sp["val_neg"].shape == sp["val_pos"].shape and sp["test_neg"].shape == sp["test_pos"].shape
    for k in ("val_neg", "test_neg"):
        assert float(d.dense_adj[sp[k][0], sp[k][1]].sum()) == 0.0
    held = set(map(tuple, torch.cat([sp["val_pos"], sp["test_pos"]], 1).t().tolist()))
    train = set(map(tuple, sp["train_pos"].t().tolist()))
    assert not (held & train)
    n = 130
    a = torch.rand(n, n, generator=torch.Generator().manual_seed(1)) < 0.1
    b = edges_to_bits(a.nonzero().t(), n, "cpu").numpy().view(np.uint64)
    cols = np.arange(n)
    dec = ((b[:, cols // 64] >> (cols % 64).astype(np.uint64)) & np.uint64(1)).astype(bool)
    assert np.array_equal(dec, a.numpy())
