"""Planetoid (Cora / Citeseer) without unpickling.

The reference loads its datasets through torch_geometric 1.3.2's `Planetoid`
(src/data/utils.py:75-78 -> torch_geometric.io.read_planetoid_data), which
unpickles the `ind.<name>.{x,tx,allx,y,ty,ally,graph}` files of Yang et al.'s
split (Python-2 pickles of scipy CSR matrices, numpy arrays and a
defaultdict).  Unpickling executes code named by the file, so this module
never does: `read_pickle_data` walks the opcode stream with
`pickletools.genops` (a parser) and interprets only data opcodes.  The
callables a pickle names (GLOBAL) stay inert symbols; the few object kinds
these files contain are rebuilt here from their pickled STATE by rules that
know their layout:

  numpy.core.multiarray._reconstruct + BUILD(version, shape, dtype, fortran, raw)
      -> np.frombuffer(raw, dtype).reshape(shape)
  numpy.dtype REDUCE(('f4' | 'i8' | ..., 0, 1)) + BUILD((3, '<' | '|', ...))
  scipy.sparse.csr.csr_matrix NEWOBJ + BUILD({'indptr', 'indices', 'data', '_shape'})
      -> Csr(indptr, indices, data, shape)
  collections.defaultdict REDUCE((list,)) + SETITEMS -> dict

Assembly then follows torch_geometric 1.3.2 `read_planetoid_data` (restated,
the library is absent here): x = [allx; tx], y = argmax([ally; ty]), the test
rows permuted into `test.index` order, Citeseer's isolated test nodes padded
with zero rows, train = first len(y) nodes, val = the next 500, test = the
test index; edges from the adjacency dict with self-loops removed and
duplicates coalesced.  `load_planetoid_npz` reads the committed fixture
(tests/golden/planetoid_<name>.npz, made by tools/make_planetoid_fixtures.py
from the reference's tst/res files) and applies the reference's default
transform chain for the Planetoid split (src/data/dataloader.py:91-113:
CreateDenseAdjacencyMatrix, NormalizeFeatures, MakeUndirected).
"""
from __future__ import annotations

import os
import pickletools
from collections import namedtuple
from typing import Any, Dict

import numpy as np
import torch

from ..utils.graph import DenseData

Csr = namedtuple("Csr", "indptr indices data shape")


class _Global:
    def __init__(self, module: str, name: str):
        self.qual = f"{module}.{name}"

    def __repr__(self):
        return f"<global {self.qual}>"


class _Call:
    """An object a pickle would build by calling `fn(*args)`; never called."""

    def __init__(self, fn: _Global, args: tuple):
        self.fn, self.args, self.state = fn, args, None
        self.items: Dict[Any, Any] = {}


_MARK = object()


def read_pickle_data(data: bytes) -> Any:
    """Interpret the data opcodes of a protocol-0..2 pickle; returns symbolic
    objects (_Call / dict / list / tuple / bytes / numbers).  Raises on any
    opcode outside the supported data subset."""
    stack: list = []
    memo: Dict[int, Any] = {}

    def pop_mark():
        i = len(stack) - 1
        while stack[i] is not _MARK:
            i -= 1
        items = stack[i + 1:]
        del stack[i:]
        return items

    for op, arg, _pos in pickletools.genops(data):
        name = op.name
        if name in ("PROTO", "FRAME"):
            continue
        if name == "STOP":
            break
        if name == "MARK":
            stack.append(_MARK)
        elif name in ("BININT", "BININT1", "BININT2", "LONG1", "LONG4", "INT", "LONG", "BINFLOAT", "FLOAT"):
            stack.append(arg)
        elif name in ("SHORT_BINSTRING", "BINSTRING", "STRING"):
            stack.append(arg.encode("latin-1") if isinstance(arg, str) else arg)  # Python-2 str = bytes
        elif name in ("BINUNICODE", "SHORT_BINUNICODE", "UNICODE", "BINBYTES", "SHORT_BINBYTES"):
            stack.append(arg)
        elif name == "NONE":
            stack.append(None)
        elif name == "NEWTRUE":
            stack.append(True)
        elif name == "NEWFALSE":
            stack.append(False)
        elif name == "EMPTY_TUPLE":
            stack.append(())
        elif name in ("TUPLE1", "TUPLE2", "TUPLE3"):
            k = {"TUPLE1": 1, "TUPLE2": 2, "TUPLE3": 3}[name]
            t = tuple(stack[-k:])
            del stack[-k:]
            stack.append(t)
        elif name == "TUPLE":
            stack.append(tuple(pop_mark()))
        elif name == "EMPTY_LIST":
            stack.append([])
        elif name == "EMPTY_DICT":
            stack.append({})
        elif name == "APPEND":
            v = stack.pop()
            stack[-1].append(v)
        elif name == "APPENDS":
            items = pop_mark()
            stack[-1].extend(items)
        elif name in ("SETITEM", "SETITEMS"):
            items = [stack.pop(), stack.pop()][::-1] if name == "SETITEM" else pop_mark()
            target = stack[-1]
            d = target.items if isinstance(target, _Call) else target
            for i in range(0, len(items), 2):
                d[items[i]] = items[i + 1]
        elif name in ("BINPUT", "LONG_BINPUT", "PUT"):
            memo[int(arg)] = stack[-1]
        elif name in ("BINGET", "LONG_BINGET", "GET"):
            stack.append(memo[int(arg)])
        elif name == "GLOBAL":
            module, _, attr = arg.partition(" ")
            stack.append(_Global(module, attr))
        elif name == "REDUCE":
            args = stack.pop()
            fn = stack.pop()
            stack.append(_Call(fn, args))
        elif name == "NEWOBJ":
            args = stack.pop()
            cls = stack.pop()
            stack.append(_Call(cls, args))
        elif name == "BUILD":
            state = stack.pop()
            stack[-1].state = state
        else:
            raise ValueError(f"pickle opcode {name} is outside the data subset this reader interprets")
    if len(stack) != 1:
        raise ValueError("malformed pickle stream")
    return stack[0]


def _dtype(node: _Call) -> np.dtype:
    if not (isinstance(node, _Call) and node.fn.qual == "numpy.dtype"):
        raise ValueError(f"expected a numpy dtype, got {node!r}")
    code = node.args[0].decode() if isinstance(node.args[0], bytes) else node.args[0]
    order = "<"
    if node.state is not None and len(node.state) > 1:
        o = node.state[1]
        order = o.decode() if isinstance(o, bytes) else o
    dt = np.dtype(code)
    return dt.newbyteorder(order) if order in "<>" else dt


def materialize(node: Any) -> Any:
    """Rebuild the supported object kinds from a read_pickle_data tree."""
    if isinstance(node, _Call):
        q = node.fn.qual
        if q == "numpy.core.multiarray._reconstruct":
            _ver, shape, dt, fortran, raw = node.state
            arr = np.frombuffer(raw if isinstance(raw, bytes) else bytes(raw), dtype=_dtype(dt))
            return arr.reshape(shape, order="F" if fortran else "C").astype(arr.dtype.newbyteorder("="))
        if q in ("scipy.sparse.csr.csr_matrix", "scipy.sparse._csr.csr_matrix"):
            st = {k.decode() if isinstance(k, bytes) else k: v for k, v in node.state.items()}
            shape = st.get("_shape", st.get("shape"))
            return Csr(materialize(st["indptr"]), materialize(st["indices"]), materialize(st["data"]),
                       tuple(int(x) for x in shape))
        if q == "collections.defaultdict":
            return {k: materialize(v) for k, v in node.items.items()}
        raise ValueError(f"object kind {q} is not rebuilt by this reader")
    if isinstance(node, list):
        return [materialize(v) for v in node]
    if isinstance(node, tuple):
        return tuple(materialize(v) for v in node)
    if isinstance(node, dict):
        return {k: materialize(v) for k, v in node.items()}
    return node


def _dense(m) -> np.ndarray:
    if isinstance(m, Csr):
        out = np.zeros(m.shape, dtype=np.float32)
        for r in range(m.shape[0]):
            a, b = int(m.indptr[r]), int(m.indptr[r + 1])
            out[r, m.indices[a:b]] = m.data[a:b]
        return out
    return np.asarray(m, dtype=np.float32)


def read_planetoid_raw(raw_dir: str, name: str) -> Dict[str, np.ndarray]:
    """torch_geometric 1.3.2 read_planetoid_data, restated on the data-only
    reader.  Returns x (float32 dense), y (int64), edge_index (2 × E int64,
    coalesced, no self-loops), train/val/test masks (bool)."""
    objs = {}
    for part in ("x", "tx", "allx", "y", "ty", "ally", "graph"):
        with open(os.path.join(raw_dir, f"ind.{name}.{part}"), "rb") as f:
            objs[part] = materialize(read_pickle_data(f.read()))
    with open(os.path.join(raw_dir, f"ind.{name}.test.index")) as f:
        test_index = np.array([int(line) for line in f if line.strip()], dtype=np.int64)
    tx, ty = _dense(objs["tx"]), np.asarray(objs["ty"], dtype=np.float32)
    allx, ally = _dense(objs["allx"]), np.asarray(objs["ally"], dtype=np.float32)
    y_train = np.asarray(objs["y"])
    sorted_test = np.sort(test_index)
    if name.lower() == "citeseer":  # isolated test nodes: zero feature / label rows
        span = int(test_index.max() - test_index.min()) + 1
        tx_ext = np.zeros((span, tx.shape[1]), dtype=np.float32)
        tx_ext[sorted_test - test_index.min()] = tx
        ty_ext = np.zeros((span, ty.shape[1]), dtype=np.float32)
        ty_ext[sorted_test - test_index.min()] = ty
        tx, ty = tx_ext, ty_ext
    x = np.concatenate([allx, tx], 0)
    y = np.concatenate([ally, ty], 0).argmax(1).astype(np.int64)  # torch .max(dim=1)[1]: first max
    x[test_index] = x[sorted_test]
    y[test_index] = y[sorted_test]
    n = y.shape[0]
    train = np.zeros(n, dtype=bool)
    train[: y_train.shape[0]] = True
    val = np.zeros(n, dtype=bool)
    val[y_train.shape[0]: y_train.shape[0] + 500] = True
    test = np.zeros(n, dtype=bool)
    test[test_index] = True
    row, col = [], []
    for key, value in objs["graph"].items():
        row += [int(key)] * len(value)
        col += [int(v) for v in value]
    e = np.array([row, col], dtype=np.int64)
    e = e[:, e[0] != e[1]]  # remove_self_loops
    e = np.unique(e[0] * n + e[1])  # coalesce: sorted by (row, col), duplicates merged
    edge_index = np.stack([e // n, e % n])
    return dict(x=x, y=y, edge_index=edge_index, train_mask=train, val_mask=val, test_mask=test)


FIXTURE_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))))), "tests", "golden")


def load_planetoid_npz(name: str = "cora", path: str = None, normalize_features: bool = True,
                       make_undirected: bool = True) -> DenseData:
    """The Planetoid split of `name` as the reference's data pipeline yields it
    for the final LDS configuration (src/data/dataloader.py:54-113 with
    shuffle_splits=False, nearest_neighbor_k=None)."""
    path = path or os.path.join(FIXTURE_DIR, f"planetoid_{name}.npz")
    z = np.load(path)  # allow_pickle=False (default): plain arrays only
    n, f = (int(v) for v in z["x_shape"])
    x = torch.sparse_csr_tensor(torch.from_numpy(z["x_indptr"]).long(), torch.from_numpy(z["x_indices"]).long(),
                                torch.from_numpy(z["x_data"]), size=(n, f)).to_dense()
    if normalize_features:  # torch_geometric NormalizeFeatures: x / x.sum(-1).clamp(min=1)
        x = x / x.sum(-1, keepdim=True).clamp(min=1)
    ei = torch.from_numpy(z["edge_index"]).long()
    adj = torch.zeros(n, n)
    adj[ei[0], ei[1]] = 1.0  # CreateDenseAdjacencyMatrix
    if make_undirected:  # MakeUndirected (src/data/transforms.py:31-37)
        adj = torch.maximum(adj, adj.t())
    y = torch.from_numpy(z["y"]).long()
    return DenseData(x=x, y=y, dense_adj=adj, train_mask=torch.from_numpy(z["train_mask"]),
                     val_mask=torch.from_numpy(z["val_mask"]), test_mask=torch.from_numpy(z["test_mask"]),
                     num_classes=int(y.max()) + 1, name=name)
