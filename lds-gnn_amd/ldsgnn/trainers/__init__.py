"""Trainers of the bilevel problem (src/trainers/)."""
from typing import NamedTuple


class Metrics(NamedTuple):
    """src/trainers/__init__.py:1-5"""
    loss: float
    acc: float
