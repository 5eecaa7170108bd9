"""Keyed randomness for the hot path.

The reference draws graph samples and dropout masks from torch's global
mt19937 stream (src/models/sampling.py:68, src/models/gcn.py:27,29), so a
result depends on every draw made before it.  Here every draw is a pure
function of (seed, tag, counter, element) — Philox4x32-10, include/ldsgnn.h
"RNG contract" — so GPU kernels can generate any element anywhere, replicas on
different GPUs get independent streams by tag, and the CPU oracle reproduces
the exact edge sets and masks.

Schedule (mirrored by oracle/lds_oracle.py:Randomness):
  * every graph sample takes the next `graph` counter, tag TAG_GRAPH | replica;
  * every training-mode forward with dropout > 0 takes the next `forward`
    counter; its two dropout sites use TAG_DROP_X / TAG_DROP_H | replica.
"""
from __future__ import annotations

from typing import Optional

TAG_GRAPH = 1 << 24
TAG_DROP_X = 2 << 24
TAG_DROP_H = 3 << 24


def tag_for(kind: int, replica: int) -> int:
    return (kind | (replica & 0xFFFFFF)) & 0xFFFFFFFF


class Generator:
    """Seed + replica + the two draw counters."""

    def __init__(self, seed: int = 0, replica: int = 0):
        self.manual_seed(seed, replica)

    def manual_seed(self, seed: int, replica: Optional[int] = None) -> "Generator":
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        if replica is not None:
            self.replica = int(replica)
        self.graph_counter = 0
        self.forward_counter = 0
        return self

    def next_graph(self) -> tuple:
        c = self.graph_counter
        self.graph_counter += 1
        return self.seed, tag_for(TAG_GRAPH, self.replica), c

    def next_forward(self) -> int:
        c = self.forward_counter
        self.forward_counter += 1
        return c

    def dropout_key(self, site: int, counter: int) -> tuple:
        return self.seed, tag_for(site, self.replica), counter

    def get_state(self) -> dict:
        return dict(seed=self.seed, replica=self.replica, graph_counter=self.graph_counter,
                    forward_counter=self.forward_counter)

    def set_state(self, state: dict) -> None:
        self.seed = state["seed"]
        self.replica = state["replica"]
        self.graph_counter = state["graph_counter"]
        self.forward_counter = state["forward_counter"]


default_generator = Generator(0, 0)


def manual_seed(seed: int, replica: Optional[int] = None) -> Generator:
    return default_generator.manual_seed(seed, replica)
