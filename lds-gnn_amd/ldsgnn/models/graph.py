"""Graph generative models (src/models/graph.py:16-78): the LDS Bernoulli model.

BernoulliGraphModel keeps θ exactly as the reference does — a Parameter holding
the row-major upper triangle incl. the diagonal (get_triu_values of the
initial adjacency) — but `sample()` never builds the dense P: it calls the
fused θ -> CSR sampler (Sampler.sample_triu).  `forward()` still returns the
dense symmetric P for API parity/inspection.

PairwiseEmbeddingSampler and GraphProposalNetwork (src/models/graph.py:81-200,
SURVEY §8(f) item 4): P comes from node embeddings (σ(E·Eᵀ), or the affine /
sigmoid / tanh / clamp of a GCN's similarity matrix) as dense torch ops —
E·Eᵀ is the rocBLAS GEMM — and is sampled by the same HIP sampler from its
upper triangle, with the KNN / EPS sparsification of the draw as a keep mask.
The straight-through gradient reaches P's upper triangle through the
sampled graph's θ-gradient assembly, and autograd carries it on to E.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Dict

import torch
from torch import Tensor, nn
from torch.nn import Parameter

from .. import rng as _rng
from ..utils.graph import cosine_similarity, get_triu_values, is_square_matrix, num_nodes_from_triu_shape, \
    triu_values_to_symmetric_matrix
from .gcn import MetaDenseGCN
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


class PairwiseEmbeddingSampler(GraphGenerativeModel):
    """src/models/graph.py:81-112: P = σ(E·Eᵀ)^prob_pow."""

    def __init__(self, n_nodes: int, embedding_dim: int, prob_pow: float = 1.0, init_bounds: float = 0.001,
                 generator: "_rng.Generator" = None):
        super().__init__()
        self.embeddings = Parameter(torch.empty((n_nodes, embedding_dim)), requires_grad=True)
        self.prob_pow = prob_pow
        self.n_edges = n_nodes ** 2
        self.init_bounds = init_bounds
        self.generator = generator
        self.reset_embeddings()

    def reset_embeddings(self):
        self.embeddings.data.uniform_(-self.init_bounds, self.init_bounds)

    def forward(self, *args, **kwargs) -> Tensor:
        return torch.sigmoid(self.embeddings @ self.embeddings.t()) ** self.prob_pow

    def sample(self, *args, **kwargs):
        return Sampler.sample(self.forward(), embeddings=self.embeddings, generator=self.generator)

    def statistics(self) -> Dict[str, float]:
        with torch.no_grad():
            total = self.forward().sum().item()
        return {"expected_num_edges": total, "percentage_edges_expected": total / self.n_edges}


class GraphProposalNetwork(GraphGenerativeModel):
    """src/models/graph.py:115-200: a GCN embeds the nodes, P = clamp(
    [tanh|σ](factor · sim(E) + bias) [+ A], 0, 1) with sim the cosine or the
    dot-product similarity; sample() caches (graph, embeddings) for refine()."""

    def __init__(self, features: Tensor, dense_adj, dropout: float = 0.0, add_original: bool = False,
                 embedding_dim: int = 128, probs_bias_init: float = 0.0, probs_factor_init: float = 1.0,
                 prob_power: float = 1.0, use_sigmoid: bool = True, use_tanh: bool = False,
                 normalize_similarities: bool = False, generator: "_rng.Generator" = None):
        super().__init__()
        assert features.size(0) == dense_adj.size(0)
        assert is_square_matrix(dense_adj)
        assert not (use_sigmoid and use_tanh)
        assert probs_factor_init > 0.0
        self.original_features = features
        self.original_adj = dense_adj
        self.features = features
        self.adj = dense_adj
        self.n_edges = dense_adj.size(0) * dense_adj.size(1)
        self.num_features = features.size(1)
        self.add_original = add_original
        self.prob_power = prob_power   # stored, not applied (as in the reference)
        self.use_sigmoid = use_sigmoid
        self.use_tanh = use_tanh
        self.normalize_similarities = normalize_similarities
        self.gcn = MetaDenseGCN(in_features=self.num_features, hidden_features=embedding_dim * 2,
                                out_features=embedding_dim, dropout=dropout)
        self.probs_factor = Parameter(torch.tensor(probs_factor_init), requires_grad=True)
        self.probs_bias = Parameter(torch.tensor(probs_bias_init), requires_grad=True)
        self.embeddings_cached = None
        self.adj_cached = None
        self.generator = generator

    def forward(self, *args, return_embeddings: bool = False, dropout_counter: int = None, **kwargs) -> Tensor:
        new_adj, _ = self.calculate_edges_and_embeddings(dropout_counter=dropout_counter)
        return new_adj

    def calculate_edges_and_embeddings(self, *args, dropout_counter: int = None, **kwargs):
        """`dropout_counter`: run the proposal GCN's dropout at that forward
        counter instead of drawing the next one (the fused engine recomputes
        the P of a draw it made, ldsgnn.fused)."""
        new_embeddings = self.gcn.forward_to_last_layer(self.features, self.adj, dropout_counter=dropout_counter)
        if self.normalize_similarities:
            similarity_matrix = cosine_similarity(new_embeddings, new_embeddings)
        else:
            similarity_matrix = new_embeddings @ new_embeddings.t()
        new_adj = self.probs_factor * similarity_matrix + self.probs_bias
        new_adj = torch.sigmoid(new_adj) if self.use_sigmoid else new_adj
        new_adj = torch.tanh(new_adj) if self.use_tanh else new_adj
        if self.add_original:
            orig = self.adj.to_dense() if hasattr(self.adj, "to_dense") and not torch.is_tensor(self.adj) \
                else self.adj
            new_adj = new_adj + orig
        new_adj = torch.clamp(new_adj, 0.0, 1.0)
        return new_adj, new_embeddings

    def sample(self, *args, **kwargs):
        edge_probs, embeddings = self.calculate_edges_and_embeddings()
        edges = Sampler.sample(edge_probs, embeddings=embeddings, generator=self.generator)
        self.adj_cached, self.embeddings_cached = edges, embeddings
        return edges

    def refine(self):
        if self.adj_cached is not None and self.embeddings_cached is not None:
            self.features = self.embeddings_cached
            self.adj = self.adj_cached

    def statistics(self, dropout_counter: int = None) -> Dict[str, float]:
        with torch.no_grad():
            total = self.forward(dropout_counter=dropout_counter).sum().item()
        return {"expected_num_edges": total, "percentage_edges_expected": total / self.n_edges,
                "probs_factor": self.probs_factor.item(), "probs_bias": self.probs_bias.item()}

