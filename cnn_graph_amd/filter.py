"""Functional filters, mirroring ``lib/filter.py`` (selected by name with
``getattr(filter, filter_type)`` at lib/gconv_lstm.py:59).

``cheby_conv(x, L, lmax, feat_out, K, W=None)`` -- lib/filter.py:45-95 -- runs
the same HIP kernels as ``GraphConv.chebyshev5``; W is ``[K*feat_in, feat_out]``
with row index ``fin*K + k``.  ``fourier_conv(x, L, lmax, Fout, K, W=None)`` --
lib/filter.py:30-42 -- is the spectral filter of ``GraphConv.fourier`` with W
``[M, Fout, Fin]`` and U from ``graph.fourier(L)``.  When W is None a weight is
created with ``truncated_normal(0, 0.1)`` and returned through
``<filter>.last_weight`` (the reference creates a TF variable in the current
scope).
"""
from __future__ import annotations

import weakref

import numpy as np
import torch

from . import graph as host_graph
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

_U_CACHE: dict = {}


def fourier_basis(L, device):
    """Device copy of U (eigenvectors of L in columns, lib/graph.py:148-166),
    computed once per (L object, device) like the reference's graph constant."""
    key = (id(L), str(device))
    hit = _U_CACHE.get(key)
    if hit is None:
        _, U = host_graph.fourier(L)
        hit = torch.as_tensor(np.ascontiguousarray(U, dtype=np.float32), device=device)
        _U_CACHE[key] = hit
        try:
            weakref.finalize(L, _U_CACHE.pop, key, None)
        except TypeError:
            pass
    return hit


def fourier_conv(x, L, lmax, Fout, K, W=None):
    N, M, Fin = (int(s) for s in x.shape)
    if W is None:
        W = torch.nn.Parameter(truncated_normal_(torch.empty((M, Fout, Fin), device=x.device), 0.1))
        fourier_conv.last_weight = W
    return ops.fourier_conv(x, W, fourier_basis(L, x.device))


fourier_conv.last_weight = None
