"""Graph sampling API (src/models/sampling.py).

The LDS configuration — undirected=True, sparsification NONE, dense=False —
is the hot path: `sample_triu` draws straight from θ (the packed upper
triangle) into CSR on the GPU (lds_sample_graph) and attaches the
straight-through gradient to θ (ldsgnn.ops).  `sample_graph` on a dense
probability matrix keeps the reference's function signature; for the
undirected case it routes through the same kernel by reading P's upper
triangle (gradients then reach P's upper triangle, which is exactly the θ
gradient when P = sym(θ)).  KNN / EPS sparsification of the Bernoulli draw
(the embedding / GAE models' option) becomes a keep-mask of the sampler:
u_ij < P_ij·keep_ij is exactly sample ⊙ keep with the same uniforms, and the
straight-through gradient still reaches every P_ij, as in the reference.
"""
from __future__ import annotations

from enum import Enum
from typing import Optional

import torch
from torch import Tensor

from .. import rng as _rng
from ..ops import SampledGraph, sample_graph_from_triu
from ..utils.graph import get_triu_values, is_square_matrix, knn_graph_dense, to_undirected


class SPARSIFICATION(Enum):
    NONE = 1
    KNN = 2
    EPS = 3


def straight_through_estimator(sample: Tensor, parameters: Tensor) -> Tensor:
    """src/models/sampling.py:82-85 (dense)."""
    assert sample.size() == parameters.size()
    return (sample - parameters).detach() + parameters


def sparsify(edge_probs: Tensor, sparsification: SPARSIFICATION, embeddings: Optional[Tensor] = None,
             k: Optional[int] = None, eps: Optional[float] = None, knn_metric: str = "cosine") -> Tensor:
    """src/models/sampling.py:19-44 on a dense matrix (probabilities or a
    sample): KNN keeps the entries of each row's k nearest neighbours in
    `embeddings` (cosine or dot, no self-loops), EPS zeroes entries < eps.
    Zeroed entries get no gradient, as in the reference."""
    if sparsification == SPARSIFICATION.NONE:
        return edge_probs
    keep = _keep_matrix(edge_probs, sparsification, embeddings, k, eps, knn_metric)
    out = edge_probs.clone()
    out[keep == 0] = 0.0
    return out


def _keep_matrix(edge_probs: Tensor, sparsification: SPARSIFICATION, embeddings: Optional[Tensor],
                 k: Optional[int], eps: Optional[float], knn_metric: str) -> Tensor:
    """The 0/1 keep pattern of sparsify (dense, edge_probs' shape)."""
    if sparsification == SPARSIFICATION.KNN:
        assert embeddings is not None, "Needs embeddings to create knn graph"
        assert k is not None and 0 < k < edge_probs.size(0)
        return knn_graph_dense(embeddings.detach(), k=k, loop=False, metric=knn_metric).to(edge_probs.device)
    if sparsification == SPARSIFICATION.EPS:
        assert eps is not None
        return (edge_probs.detach() >= eps).to(torch.float32)
    raise NotImplementedError()


def _sample_keep(n: int, device, sparsification: SPARSIFICATION, embeddings: Optional[Tensor],
                 k: Optional[int], eps: Optional[float], knn_metric: str) -> Optional[Tensor]:
    """Packed-triu keep mask for sparsifying a Bernoulli SAMPLE (0/1 values):
    KNN -> row i's kNN pattern at (i, j), i <= j (to_undirected then reads the
    upper triangle); EPS -> every sampled 1 survives iff 1 >= eps."""
    if sparsification == SPARSIFICATION.NONE:
        return None
    if sparsification == SPARSIFICATION.KNN:
        assert embeddings is not None, "Needs embeddings to create knn graph"
        assert k is not None and 0 < k < n
        knn = knn_graph_dense(embeddings.detach(), k=k, loop=False, metric=knn_metric).to(device)
        return get_triu_values(knn).contiguous()
    if sparsification == SPARSIFICATION.EPS:
        assert eps is not None
        fill = 1.0 if 1.0 >= eps else 0.0
        return torch.full((n * (n + 1) // 2,), fill, dtype=torch.float32, device=device)
    raise NotImplementedError()


def sample_graph(edge_probs: Tensor, undirected: bool, embeddings: Optional[Tensor] = None,
                 dense: bool = False, k: Optional[int] = None,
                 sparsification: SPARSIFICATION = SPARSIFICATION.NONE,
                 force_straight_through_estimator: bool = False, eps: Optional[float] = None,
                 knn_metric: str = "cosine", generator: "_rng.Generator" = None,
                 u_inject: Optional[Tensor] = None):
    """src/models/sampling.py:47-79."""
    assert is_square_matrix(edge_probs)
    assert embeddings is None or edge_probs.size(0) == embeddings.size(0)
    sp = dict(embeddings=embeddings, k=k, eps=eps, knn_metric=knn_metric)
    if dense:
        sample = sparsify(edge_probs, sparsification, **sp)
        sample = to_undirected(sample, from_triu_only=True) if undirected else sample
        return straight_through_estimator(sample, edge_probs) if force_straight_through_estimator else sample
    if undirected:
        n = edge_probs.size(0)
        keep = _sample_keep(n, edge_probs.device, sparsification, **sp)
        return sample_graph_from_triu(get_triu_values(edge_probs).contiguous(), n,
                                      generator=generator, u_inject=u_inject, keep=keep)
    # directed Bernoulli graph: dense, reference semantics (not the LDS path)
    sample = sparsify(torch.bernoulli(edge_probs.detach()), sparsification, **sp)
    return straight_through_estimator(sample, edge_probs)


class Sampler:
    """src/models/sampling.py:88-138.  `config` holds the sacred defaults
    (src/models/sampling.py:96-102) and may be edited like the ingredient."""

    config = dict(undirected=True, k=20, eps=0.9, sparsification="NONE", dense=False,
                  knn_metric="cosine")

    @staticmethod
    def sample(edge_probs: Tensor, undirected: bool = None, sparsification: str = None,
               k: int = None, eps: float = None, embeddings: Tensor = None, dense: bool = None,
               knn_metric: str = None, generator: "_rng.Generator" = None, u_inject: Optional[Tensor] = None):
        c = Sampler.config
        undirected = c["undirected"] if undirected is None else undirected
        sparsification = c["sparsification"] if sparsification is None else sparsification
        dense = c["dense"] if dense is None else dense
        assert sparsification in SPARSIFICATION.__members__
        return sample_graph(edge_probs=edge_probs, embeddings=embeddings, undirected=undirected,
                            sparsification=SPARSIFICATION[sparsification], dense=dense,
                            k=c["k"] if k is None else k, eps=c["eps"] if eps is None else eps,
                            knn_metric=c["knn_metric"] if knn_metric is None else knn_metric,
                            generator=generator, u_inject=u_inject)

    @staticmethod
    def sample_triu(theta: Tensor, n: int, generator: "_rng.Generator" = None,
                    u_inject: Optional[Tensor] = None) -> SampledGraph:
        """The LDS path: θ (packed triu) -> SampledGraph, no dense P."""
        c = Sampler.config
        if not c["undirected"] or c["dense"] or c["sparsification"] != "NONE":
            raise NotImplementedError("sample_triu implements the LDS configuration only")
        return sample_graph_from_triu(theta, n, generator=generator, u_inject=u_inject)
