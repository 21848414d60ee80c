"""Drop-in for the filter plug-in of ``lib/graph_conv.py::GraphConv`` (and the
identical ``lib/models.py::cgcnn``): the model binds its graph filter, bias /
activation and pooling by *name* (lib/graph_conv.py:74-76), so reference code
that builds layers as ``self.filter(x, L, Fout, K)`` keeps working with
``filter='chebyshev5'`` selecting the HIP kernels.

Only what the Chebyshev path needs is mirrored here: the name binding,
``tf.variable_scope``-style weight naming with ``truncated_normal(0, 0.1)``
initialisation (lib/graph_model.py:326-333), ``chebyshev5``, ``b1relu``,
``mpool1`` / ``apool1``, and the residual stack that calls them
(lib/graph_conv.py:234-330).  Everything else of the TF model class
(sessions, feeds, summaries) is outside the hot path.
"""
from __future__ import annotations

import contextlib

import torch

from . import ops
from .plan import plan_for


def truncated_normal_(t: torch.Tensor, std=0.1, generator=None):
    """tf.truncated_normal_initializer(0, std): resample |z| > 2 std."""
    with torch.no_grad():
        t.normal_(0.0, std, generator=generator)
        bad = t.abs() > 2 * std
        while bool(bad.any()):
            t[bad] = torch.empty(int(bad.sum()), device=t.device).normal_(0.0, std, generator=generator)
            bad = t.abs() > 2 * std
    return t


class GraphConv:
    """Filter plumbing of lib/graph_conv.py::GraphConv on MI355X.

    filter / brelu / pool are bound by name exactly like :74-76.  Weights are
    created on first use per variable scope (the ``tf.get_variable('weights')``
    contract of ``chebyshev5``: one ``weights`` per enclosing scope) and kept in
    ``self.weights`` ({scope/weights: Parameter}) and ``self.nets``.
    """

    def __init__(self, filter="chebyshev5", brelu="b1relu", pool="mpool1", device=None,
                 seed=2017, path="auto"):
        self.device = torch.device(device if device is not None else "cuda")
        self.filter = getattr(self, filter)
        self.brelu = getattr(self, brelu)
        self.pool = getattr(self, pool)
        self.path = path
        self.weights: dict[str, torch.nn.Parameter] = {}
        self.nets: dict[str, torch.Tensor] = {}
        self._scope: list[str] = []
        self._gen = torch.Generator(device=self.device)
        self._gen.manual_seed(seed)   # tf.set_random_seed(2017), lib/graph_model.py:41

    # -- variable scopes -------------------------------------------------------
    @contextlib.contextmanager
    def variable_scope(self, name):
        self._scope.append(name)
        try:
            yield
        finally:
            self._scope.pop()

    def _weight_variable(self, shape, regularization=True):
        name = "/".join(self._scope + ["weights"])
        w = self.weights.get(name)
        if w is None:
            w = torch.nn.Parameter(truncated_normal_(
                torch.empty(tuple(shape), device=self.device), 0.1, self._gen))
            self.weights[name] = w
            self.nets[name] = w
        elif tuple(w.shape) != tuple(shape):
            raise ValueError(f"variable {name} exists with shape {tuple(w.shape)}, asked {tuple(shape)}")
        return w

    def parameters(self):
        return list(self.weights.values())

    # -- filters ---------------------------------------------------------------
    def chebyshev5(self, x, L, Fout, K):
        """lib/graph_conv.py:144-176 on the HIP path.  x: [N, M, Fin] cuda fp32;
        L: scipy sparse normalized Laplacian; returns [N, M, Fout]."""
        N, M, Fin = (int(s) for s in x.shape)
        plan = plan_for(L, lmax=2, device=x.device.index or 0, path=self.path)
        W = self._weight_variable([Fin * K, Fout], regularization=False)
        return ops.cheb_conv(x, W, plan, int(K))

    def _filter_act(self, x, L, Fout, K, residual=None):
        """b1relu(filter(x) [+ residual]) -- fused into the filter's y store when
        the bound filter / activation are chebyshev5 / b1relu (the residual
        block's `x = filter(x)`, `x = x + x_identity`, `x = brelu(x)`,
        lib/graph_conv.py:256-262); otherwise the separate calls."""
        fuse = (getattr(self.filter, "__func__", None) is GraphConv.chebyshev5 and
                getattr(self.brelu, "__func__", None) is GraphConv.b1relu)
        if not fuse:
            y = self.filter(x, L, Fout, K)
            if residual is not None:
                y = y + residual
            return self.brelu(y)
        N, M, Fin = (int(s) for s in x.shape)
        plan = plan_for(L, lmax=2, device=x.device.index or 0, path=self.path)
        W = self._weight_variable([Fin * K, Fout], regularization=False)
        return ops.cheb_conv(x, W, plan, int(K), residual=residual, act="relu")

    # -- activations / pooling -----------------------------------------------------
    def b1relu(self, x):
        """lib/graph_conv.py:178-187 (its bias is commented out -> plain ReLU)."""
        return torch.relu(x)

    def mpool1(self, x, p):
        return ops.mpool1(x, int(p))

    def apool1(self, x, p):
        return ops.apool1(x, int(p))

    # -- the residual stack that calls the filter (lib/graph_conv.py:234-330) ----
    def residual_layer(self, x, L, nfilter, K, name_scope, residual=True):
        x_identity = x
        with self.variable_scope(name_scope):
            with self.variable_scope("sublayer0" if residual else "sublayer0nores"):
                x = self._filter_act(x, L, nfilter, K)
            with self.variable_scope("sublayer1" if residual else "sublayer1nores"):
                x = self._filter_act(x, L, nfilter, K, x_identity if residual else None)
        return x

    def residual_network(self, x, L, nfilter, K, nres_layer_count, Fout_last=2):
        with self.variable_scope("conv_init"):
            x = self._filter_act(x, L, nfilter, K)
        for i in range(nres_layer_count):
            x = self.residual_layer(x, L, nfilter, K, f"residual_layer_{i}")
        with self.variable_scope("convN"):
            x = self.filter(x, L, Fout_last, K)
        return x
