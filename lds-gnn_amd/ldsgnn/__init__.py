"""ldsgnn — MI355X-native LDS (Learning Discrete Structures) bilevel hot path.

Drop-in for the hot path of andreas-grafberger/lds-gnn: the reference's
Python API (MetaDenseGCN, BernoulliGraphModel, Sampler, Inner/Outer trainers,
BilevelProblemRunner) over hand-written HIP kernels for gfx950 (libldsgnn.so,
C-ABI in include/ldsgnn.h).  Importing this package loads the native library
and fails loudly if it is missing — there is no CPU fallback.
"""
from . import _native  # noqa: F401  (load + ABI check first)
from . import rng  # noqa: F401
from .ops import CsrGraph, SampledGraph, aggregate, csr_graph_from_dense, sample_graph_from_triu  # noqa: F401

__version__ = "0.1.0"
