"""Functional-parameter modules — the slice of torchmeta the reference uses.

The reference builds its GCN on `torchmeta==1.2.1` (environment.yml:34):
`MetaModule`, `MetaLinear` and `get_subdict` (src/models/gcn.py:2-3,
src/models/layers.py:5-6).  torchmeta is not vendored in the reference and is
not installed here; this restates its published behaviour for that slice:

  MetaLinear.forward(x, params) = F.linear(x, params['weight'], params.get('bias'))
  get_subdict(params, key)      = {k[len(key)+1:]: v for k with prefix key + '.'}
                                  (None when params is None)
"""
from __future__ import annotations

import re
from collections import OrderedDict
from typing import Optional

import torch.nn.functional as F
from torch import nn


def get_subdict(params: Optional[dict], key: Optional[str] = None):
    if params is None:
        return None
    if not key:
        return params
    key_re = re.compile(r"^{0}\.(.+)".format(re.escape(key)))
    return OrderedDict((key_re.sub(r"\1", k), v) for (k, v) in params.items() if key_re.match(k) is not None)


class MetaModule(nn.Module):
    """nn.Module whose forward accepts a `params` override dict."""

    def meta_named_parameters(self, prefix: str = "", recurse: bool = True):
        return self.named_parameters(prefix=prefix, recurse=recurse)

    def meta_parameters(self, recurse: bool = True):
        for _, p in self.meta_named_parameters(recurse=recurse):
            yield p


class MetaLinear(nn.Linear, MetaModule):
    __doc__ = nn.Linear.__doc__

    def forward(self, input, params=None):
        if params is None:
            params = OrderedDict(self.named_parameters())
        return F.linear(input, params["weight"], params.get("bias", None))
