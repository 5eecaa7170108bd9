"""Graph-model factory (src/models/factory.py).

`create("lds" | "embedding" | "gae")` and `optimizer(model)` with the
reference's ingredient defaults (src/models/factory.py:24-174) as editable
class-level dicts (sacred's config role).
"""
from __future__ import annotations

from typing import Type

from torch.optim import SGD, Adam, Optimizer

from .graph import BernoulliGraphModel, GraphGenerativeModel, GraphProposalNetwork, PairwiseEmbeddingSampler


class GraphGenerativeModelFactory:
    lds_config = dict(directed=False, lr=1.0)  # src/models/factory.py:53-56
    embedding_config = dict(embedding_dim=16, prob_pow=1.0, lr=0.1, init_bounds=0.001)  # :75-81
    gae_config = dict(dropout=0.0, add_original=False, embedding_dim=16, probs_bias_init=0.0,  # :107-121
                      probs_factor_init=1.0, prob_power=1.0, use_sigmoid=True, normalize_similarities=True,
                      weights_lr=0.01, gcn_weight_decay=0.0005, affine_prob_lr=0.01, optimizer_type="SGD",
                      use_tanh=False)

    def __init__(self, data):
        self.data = data

    def create(self, model_name: str) -> GraphGenerativeModel:
        name = model_name.lower()
        if name == "lds":
            return BernoulliGraphModel(self.data.dense_adj, directed=self.lds_config["directed"])
        dev = self.data.x.device
        if name == "embedding":
            c = self.embedding_config
            return PairwiseEmbeddingSampler(n_nodes=self.data.x.size(0), embedding_dim=c["embedding_dim"],
                                            prob_pow=c["prob_pow"], init_bounds=c["init_bounds"]).to(dev)
        if name == "gae":
            c = self.gae_config
            return GraphProposalNetwork(features=self.data.x, dense_adj=self.data.dense_adj, dropout=c["dropout"],
                                        add_original=c["add_original"], embedding_dim=c["embedding_dim"],
                                        probs_bias_init=c["probs_bias_init"],
                                        probs_factor_init=c["probs_factor_init"], prob_power=c["prob_power"],
                                        use_sigmoid=c["use_sigmoid"], use_tanh=c["use_tanh"],
                                        normalize_similarities=c["normalize_similarities"]).to(dev)
        raise NotImplementedError(f"Model {model_name} not supported.")

    def optimizer(self, model: GraphGenerativeModel) -> Optimizer:
        if type(model) == BernoulliGraphModel:
            return SGD(model.parameters(), lr=self.lds_config["lr"])
        if type(model) == PairwiseEmbeddingSampler:
            return self.embeddings_optimizer(model, lr=self.embedding_config["lr"])
        if type(model) == GraphProposalNetwork:
            c = self.gae_config
            opt_type = self.get_optimizer(c["optimizer_type"])
            affine_prob_lr = c["affine_prob_lr"] or c["weights_lr"]
            return opt_type(params=[
                {"params": model.gcn.parameters(), "weight_decay": c["gcn_weight_decay"], "lr": c["weights_lr"]},
                {"params": [model.probs_factor, model.probs_bias], "lr": affine_prob_lr}])
        raise NotImplementedError(f"Optimizer for model type {type(model)} not implemented.")

    @staticmethod
    def embeddings_optimizer(model: PairwiseEmbeddingSampler, lr: float) -> Optimizer:
        return SGD(model.parameters(), lr=lr)

    @staticmethod
    def get_optimizer(optimizer_type: str) -> Type[Optimizer]:
        if optimizer_type.lower() == "sgd":
            return SGD
        if optimizer_type.lower() == "adam":
            return Adam
        raise NotImplementedError()
