"""Graph convolution layers (src/models/layers.py:9-44).

`forward(x, graph)` computes graph·(x Wᵀ + b) — bias BEFORE aggregation, as the
reference does (src/models/layers.py:43-44).  `graph` is either a hot-path
graph (ldsgnn.ops.CsrGraph / SampledGraph: the normalised Â applied by the
lds_spmm_norm HIP kernel, differentiable in x and θ) or, with reference
semantics, a dense matrix the caller already normalised (torch.mm).
"""
from __future__ import annotations

import torch
from torch import nn
from torch.nn import Parameter
from torch.nn.init import xavier_uniform_

from ..ops import CsrGraph, aggregate
from .meta import MetaLinear, MetaModule, get_subdict


def _xavier_like(w: torch.Tensor) -> torch.Tensor:
    # Drawn from the CPU generator, as the reference does when run on CPU
    # (src/models/layers.py:38-40), then moved: identical initial weights on
    # every device for the same torch.manual_seed.
    return xavier_uniform_(w.detach().to("cpu", copy=True)).to(w.device)


def _aggregate(graph, embeddings: torch.Tensor) -> torch.Tensor:
    if isinstance(graph, CsrGraph):
        return aggregate(embeddings, graph)
    return torch.mm(graph, embeddings)


class DenseGraphConvolution(nn.Module):
    """src/models/layers.py:9-27"""

    def __init__(self, in_features, out_features, use_bias=True):
        super().__init__()
        self.fc = nn.Linear(in_features, out_features, bias=use_bias)
        self.reset_weights()

    def reset_weights(self):
        self.fc.weight = Parameter(_xavier_like(self.fc.weight))
        if self.fc.bias is not None:
            self.fc.bias = Parameter(self.fc.bias.detach().clone().zero_())

    def forward(self, node_features, dense_adj):
        return _aggregate(dense_adj, self.fc(node_features))


class MetaDenseGraphConvolution(MetaModule):
    """src/models/layers.py:30-44"""
    __doc__ = DenseGraphConvolution.__doc__

    def __init__(self, in_features, out_features, use_bias=True):
        super().__init__()
        self.fc = MetaLinear(in_features, out_features, bias=use_bias)
        self.reset_weights()

    def reset_weights(self):
        self.fc.weight = Parameter(_xavier_like(self.fc.weight))
        if self.fc.bias is not None:
            self.fc.bias = Parameter(self.fc.bias.detach().clone().zero_())

    def forward(self, node_features, dense_adj, params=None):
        embeddings = self.fc.forward(node_features, params=get_subdict(params, "fc"))
        return _aggregate(dense_adj, embeddings)
