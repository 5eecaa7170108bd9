"""Patience-based stopping rule of the reference
(src/utils/early_stopping.py:7-39), restated.

Rule, per `update(value)` call number t (0-based):
- during the grace period (t <= patience) the value is always accepted;
- afterwards it is accepted iff it is <= the mean of the `patience` values
  recorded just before it (an empty window never accepts);
- a rejected value sets `abort`; so does reaching t >= max_epochs;
- an accepted value snapshots the model's state_dict and/or the given
  parameters (the "best" model the runner restores).

The mean is numpy's float64 mean over the recorded values, as in the
reference, so ties are decided the same way.  Pinned by the reference KATs in
tests/test_oracle_golden.py and the golden stopping epochs.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Union

import numpy as np
import torch


class EarlyStopping:

    def __init__(self, patience: int, max_epochs: int = 10000):
        self.patience = patience
        self.max_epochs = max_epochs
        self.losses: List[float] = []
        self.curr_step = 0
        self.abort = False
        self.model_state_dict: Optional[Dict] = None
        self.model_params = None

    def _accepts(self, value) -> bool:
        if self.curr_step <= self.patience:
            return True
        end = len(self.losses) - 1  # `value` is the last entry
        window = self.losses[max(0, end - self.patience):end]
        return len(window) > 0 and bool(value <= np.mean(window))

    def update(self, new_value, model: torch.nn.Module = None,
               model_params: Union[Dict, torch.Tensor, List] = None):
        self.losses.append(new_value)
        if not self._accepts(new_value):
            self.abort = True
        else:
            if model is not None:
                self.model_state_dict = model.state_dict()
            if model_params is not None:
                self.model_params = model_params
        self.abort = self.abort or self.curr_step >= self.max_epochs
        self.curr_step += 1

    def best_model_state_dict(self):
        return self.model_state_dict
