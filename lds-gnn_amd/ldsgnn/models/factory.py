"""Graph-model factory (src/models/factory.py), LDS branch only.

`create("lds")` -> BernoulliGraphModel(data.dense_adj); `optimizer` -> SGD(lr)
(src/models/factory.py:24-69).  "embedding" / "gae" are out of scope.
"""
from __future__ import annotations

from torch.optim import SGD, Optimizer

from .graph import BernoulliGraphModel, GraphGenerativeModel


class GraphGenerativeModelFactory:
    lds_config = dict(directed=False, lr=1.0)  # src/models/factory.py:53-56

    def __init__(self, data):
        self.data = data

    def create(self, model_name: str) -> GraphGenerativeModel:
        name = model_name.lower()
        if name == "lds":
            return BernoulliGraphModel(self.data.dense_adj, directed=self.lds_config["directed"])
        raise NotImplementedError(f"Model {model_name} not supported.")

    def optimizer(self, model: GraphGenerativeModel) -> Optimizer:
        if type(model) == BernoulliGraphModel:
            return SGD(model.parameters(), lr=self.lds_config["lr"])
        raise NotImplementedError(f"Optimizer for model type {type(model)} not implemented.")
