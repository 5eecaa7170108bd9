"""The bilevel control loop (src/trainers/bilevel.py:17-145).

Same loop, counters and early-stopping rules as the reference; sacred's
`Run.log_scalar` becomes an optional `logger(name, value, step)` callable
(JSON-lines in scripts).  `current_step` is global across outer epochs and a
hyper step runs iff `hyper_gradient_interval == 0 or step % τ == 0`.
"""
from __future__ import annotations

import logging
from copy import deepcopy
from typing import Callable, Dict, Optional

from ..utils.early_stopping import EarlyStopping
from ..utils.evaluation import empirical_mean_loss
from . import Metrics
from .inner import InnerProblemTrainer
from .outer import OuterProblemTrainer

Logger = Callable[[str, float, Optional[int]], None]


class BilevelProblemRunner:

    def __init__(self, inner_trainer: InnerProblemTrainer, outer_trainer: OuterProblemTrainer, data,
                 n_samples_empirical_mean: int = 16):
        self.inner_trainer = inner_trainer
        self.outer_trainer = outer_trainer
        self.data = data
        self.gcn_params = None
        self.graph_state_dict = None
        self.n_samples_empirical_mean = n_samples_empirical_mean
        self.logger = logging.getLogger("ldsgnn.bilevel")

    def train(self, patience: int, hyper_gradient_interval: int, inner_loop_max_epochs: int = 400,
              outer_loop_max_epochs: int = 400, sacred_runner: Optional[Logger] = None):
        log = sacred_runner
        outer_early_stopper = EarlyStopping(patience=patience, max_epochs=outer_loop_max_epochs)
        current_step = 0
        outer_step = 0
        while not outer_early_stopper.abort:
            inner_early_stopper = EarlyStopping(patience=patience, max_epochs=inner_loop_max_epochs)
            self.inner_trainer.reset_weights()
            self.inner_trainer.reset_optimizer()
            while not inner_early_stopper.abort:
                m = self.inner_opt_step()
                inner_early_stopper.update(m.loss, model_params=self.inner_trainer.copy_model_params())
                if log is not None:
                    log("loss.train", m.loss, current_step)
                    log("acc.train", m.acc, current_step)
                if hyper_gradient_interval == 0 or current_step % hyper_gradient_interval == 0:
                    self.hyper_opt_step(current_step, log)
                current_step += 1
            gcn_model_params = inner_early_stopper.model_params
            self.outer_trainer.train(False)
            val, test = empirical_mean_loss(self.inner_trainer.model, graph_model=self.outer_trainer.model,
                                            n_samples=self.n_samples_empirical_mean, data=self.data,
                                            model_parameters=gcn_model_params)
            if log is not None:
                log("loss.val.empirical", val.loss, None)
                log("acc.val.empirical", val.acc, None)
                log("loss.test.empirical", test.loss, None)
                log("acc.test.empirical", test.acc, None)
            outer_early_stopper.update(val.loss, model_params=[deepcopy(gcn_model_params),
                                                                self.outer_trainer.model.state_dict()])
            outer_step += 1
        self.logger.info("Ended training after %d steps...", outer_step)
        self.gcn_params, self.graph_state_dict = outer_early_stopper.model_params

    def inner_opt_step(self) -> Metrics:
        self.outer_trainer.train()
        graph = self.outer_trainer.sample()
        return self.inner_trainer.train_step(graph)

    def hyper_opt_step(self, current_step: int, sacred_runner: Optional[Logger] = None):
        metrics = self.outer_trainer.train_step(self.inner_trainer.model_forward)
        self.inner_trainer.detach()
        self.outer_trainer.detach()
        if sacred_runner is not None:
            sacred_runner("loss.outer", metrics.loss, current_step)
            sacred_runner("acc.outer", metrics.acc, current_step)
            for i, lr in enumerate(self.outer_trainer.get_learning_rates()):
                sacred_runner(f"Outer Learning Rate {i}", lr, current_step)
            for name, value in self.outer_trainer.model.statistics().items():
                sacred_runner(name, value, current_step)
        return metrics

    def evaluate(self) -> Dict:
        assert self.gcn_params is not None and self.graph_state_dict is not None, \
            "Models need to be trained before evaluation."
        self.outer_trainer.model.load_state_dict(self.graph_state_dict)
        val, test = empirical_mean_loss(self.inner_trainer.model, graph_model=self.outer_trainer.model,
                                        n_samples=self.n_samples_empirical_mean, data=self.data,
                                        model_parameters=self.gcn_params)
        return {"loss.val.final": val.loss, "acc.val.final": val.acc,
                "loss.test.final": test.loss, "acc.test.final": test.acc}
