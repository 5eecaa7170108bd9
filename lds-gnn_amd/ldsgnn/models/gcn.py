"""2-layer dense-API GCN (src/models/gcn.py:9-34).

forward(x, graph, params) = log_softmax(Â·(drop(relu(Â·(drop(x)W0ᵀ + b0)))W1ᵀ + b1))

With a hot-path graph (ldsgnn.ops.CsrGraph / SampledGraph) normalisation is
implicit in the graph (s = deg^-1/2, self-loops set) and both aggregations run
on the lds_spmm_norm HIP kernel; dropout is keyed (ldsgnn.rng) and runs on the
lds_dropout kernel.  A fixed symmetric 0/1 adjacency on the device (the
dataset graph of BASELINE config 1) is converted once to that CSR form
(`fixed_graph`); any other dense tensor graph keeps the reference semantics
(normalize_adjacency_matrix + torch.mm) on its device.
"""
from __future__ import annotations

import weakref

import torch
import torch.nn.functional as F

from .. import rng as _rng
from ..ops import CsrGraph, csr_graph_from_dense, keyed_dropout
from ..utils.graph import normalize_adjacency_matrix
from .layers import MetaDenseGraphConvolution
from .meta import MetaModule, get_subdict

_FIXED: list = []  # [(weakref to the adjacency, its version, CsrGraph | None)], most recent last


def fixed_graph(adj: torch.Tensor):
    """The hot-path CSR form of a fixed dense adjacency, or None when the
    dense semantics must stay: CPU tensors, adjacencies that carry a gradient,
    and anything that is not a symmetric 0/1 matrix (the diagonal is ignored:
    self-loops are set, src/utils/graph.py:123-133).  Cached per
    tensor object and version (in-place edits invalidate), last 8 entries."""
    if not isinstance(adj, torch.Tensor) or not adj.is_cuda or adj.requires_grad or adj.dim() != 2 \
            or adj.size(0) != adj.size(1):
        return None
    for i, (ref, version, graph) in enumerate(_FIXED):
        if ref() is adj and version == adj._version:
            _FIXED.append(_FIXED.pop(i))
            return graph
    a = adj.detach()
    off = a.clone()
    off.fill_diagonal_(0.0)
    ok = bool(((off == 0) | (off == 1)).all()) and torch.equal(off, off.t())
    graph = csr_graph_from_dense(a) if ok else None
    _FIXED[:] = [e for e in _FIXED if e[0]() is not None and e[0]() is not adj][-7:]
    _FIXED.append((weakref.ref(adj), adj._version, graph))
    return graph


class MetaDenseGCN(MetaModule):

    def __init__(self, in_features, hidden_features, out_features, dropout, normalize_adj: bool = True,
                 generator: "_rng.Generator" = None):
        super().__init__()
        self.layer_in = MetaDenseGraphConvolution(in_features, hidden_features)
        self.layer_out = MetaDenseGraphConvolution(hidden_features, out_features)
        self.dropout = dropout
        self.normalize_adj = normalize_adj
        self.generator = generator  # None -> ldsgnn.rng.default_generator

    def reset_weights(self):
        self.layer_in.reset_weights()
        self.layer_out.reset_weights()

    def _dropout_keys(self, counter: int = None):
        """Keys of this forward's two dropout sites: the generator's next
        forward counter, or `counter` when given (a replayed forward — the
        fused engine's per-draw GAE proposals — takes no new counter)."""
        if not self.training or self.dropout == 0.0:
            return None, None
        gen = self.generator or _rng.default_generator
        c = gen.next_forward() if counter is None else int(counter)
        return gen.dropout_key(_rng.TAG_DROP_X, c), gen.dropout_key(_rng.TAG_DROP_H, c)

    def _drop(self, x, key):
        if key is None:
            return x
        return keyed_dropout(x, self.dropout, key)  # HIP kernel; raises for CPU tensors

    def forward_to_last_layer(self, node_features, dense_adj, params=None, dropout_counter: int = None):
        if isinstance(dense_adj, CsrGraph):
            if not self.normalize_adj:
                raise NotImplementedError("hot-path graphs are normalised by construction "
                                          "(normalize_adj=False needs a dense graph)")
        elif self.normalize_adj:
            # a fixed symmetric 0/1 device adjacency (the dataset graph, BASELINE
            # config 1: src/scripts/gcn.py:78) runs on the hot path as a cached
            # CSR graph; anything else keeps the reference's dense semantics
            graph = fixed_graph(dense_adj)
            dense_adj = graph if graph is not None else normalize_adjacency_matrix(dense_adj)
        kx, kh = self._dropout_keys(dropout_counter)
        embeddings = self._drop(node_features, kx)
        embeddings = F.relu(self.layer_in(embeddings, dense_adj, params=get_subdict(params, "layer_in")))
        embeddings = self._drop(embeddings, kh)
        return self.layer_out(embeddings, dense_adj, params=get_subdict(params, "layer_out"))

    def forward(self, node_features, dense_adj, params=None):
        embeddings = self.forward_to_last_layer(node_features, dense_adj, params=params)
        return F.log_softmax(embeddings, dim=1)
