"""Graph generative models (src/models/graph.py:16-78): the LDS Bernoulli model.

BernoulliGraphModel keeps θ exactly as the reference does — a Parameter holding
the row-major upper triangle incl. the diagonal (get_triu_values of the
initial adjacency) — but `sample()` never builds the dense P: it calls the
fused θ -> CSR sampler (Sampler.sample_triu).  `forward()` still returns the
dense symmetric P for API parity/inspection.  PairwiseEmbeddingSampler and
GraphProposalNetwork (the report's GAE models) are out of scope.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Dict

import torch
from torch import Tensor, nn
from torch.nn import Parameter

from .. import rng as _rng
from ..utils.graph import get_triu_values, is_square_matrix, num_nodes_from_triu_shape, \
    triu_values_to_symmetric_matrix
from .sampling import Sampler


class ParameterClamper(object):
    """src/models/graph.py:16-20"""

    def __call__(self, module):
        for param in module.parameters():
            param.data.clamp_(0.0, 1.0)


class GraphGenerativeModel(nn.Module, ABC):
    """src/models/graph.py:23-42"""

    def __init__(self, sample_undirected: bool = True, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.sample_undirected = sample_undirected

    def sample(self, *args, **kwargs):
        return Sampler.sample(self.forward())

    def project_parameters(self):
        pass

    def refine(self):
        pass

    @abstractmethod
    def statistics(self) -> Dict[str, float]:
        pass


class BernoulliGraphModel(GraphGenerativeModel):
    """src/models/graph.py:45-78"""

    def __init__(self, init_matrix: Tensor, directed: bool = False,
                 generator: "_rng.Generator" = None):
        super().__init__()
        assert is_square_matrix(init_matrix)
        self.directed = directed
        self.orig_matrix = init_matrix
        probs = init_matrix if directed else get_triu_values(init_matrix)
        self.probs = Parameter(probs.detach().clone().float().contiguous(), requires_grad=True)
        self.generator = generator  # None -> ldsgnn.rng.default_generator

    @property
    def num_nodes(self) -> int:
        return self.probs.size(0) if self.directed else num_nodes_from_triu_shape(self.probs.numel())

    def project_parameters(self):
        self.apply(ParameterClamper())

    def forward(self, *args, **kwargs) -> Tensor:
        return self.probs if self.directed else triu_values_to_symmetric_matrix(self.probs)

    def sample(self, *args, **kwargs):
        if self.directed:
            return Sampler.sample(self.forward(), generator=self.generator)
        return Sampler.sample_triu(self.probs, self.num_nodes, generator=self.generator)

    def statistics(self) -> Dict[str, float]:
        """Same keys as src/models/graph.py:69-78, computed from θ (no N² P)."""
        with torch.no_grad():
            if self.directed:
                p = self.probs.clamp(0.0, 1.0)
                total = p.sum()
                n = p.size(0)
            else:
                n = self.num_nodes
                t = self.probs.clamp(0.0, 1.0)
                idx = torch.arange(n, device=t.device)
                diag = t[idx * (2 * n - idx + 1) // 2]
                total = 2.0 * t.sum() - diag.sum()
            vals = torch.stack([total.double(), torch.mean(self.probs).double(),
                                torch.min(self.probs).double(), torch.max(self.probs).double()]).tolist()
        n_edges = n ** 2
        return {"expected_num_edges": vals[0], "percentage_edges_expected": vals[0] / n_edges,
                "mean_prob": vals[1], "min_prob": vals[2], "max_prob": vals[3]}
