"""Functional filters, mirroring ``lib/filter.py`` (selected by name with
``getattr(filter, filter_type)`` at lib/gconv_lstm.py:59).

``cheby_conv(x, L, lmax, feat_out, K, W=None)`` -- lib/filter.py:45-95 -- runs
the same HIP kernels as ``GraphConv.chebyshev5``; W is ``[K*feat_in, feat_out]``
with row index ``fin*K + k``.  When W is None a weight is created with
``truncated_normal(0, 0.1)`` and returned through ``cheby_conv.last_weight``
(the reference creates a TF variable in the current scope).
"""
from __future__ import annotations

import torch

from . import ops
from .graph_conv import truncated_normal_
from .plan import plan_for


def cheby_conv(x, L, lmax, feat_out, K, W=None):
    N, M, Fin = (int(s) for s in x.shape)
    if W is None:
        W = torch.nn.Parameter(truncated_normal_(torch.empty((K * Fin, feat_out), device=x.device), 0.1))
        cheby_conv.last_weight = W
    plan = plan_for(L, lmax=lmax, device=x.device.index or 0)
    return ops.cheb_conv(x, W, plan, int(K))


cheby_conv.last_weight = None
