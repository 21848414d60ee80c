"""Drop-in for the filter plug-in of ``lib/graph_conv.py::GraphConv`` (and the
identical ``lib/models.py::cgcnn``): the model binds its graph filter, bias /
activation and pooling by *name* (lib/graph_conv.py:74-76), so reference code
that builds layers as ``self.filter(x, L, Fout, K)`` keeps working with
``filter='chebyshev5'`` selecting the HIP kernels.

Mirrored here: the name binding, ``tf.variable_scope``-style variable naming
with ``truncated_normal(0, 0.1)`` weights and ``constant(0.1)`` biases
(lib/graph_model.py:326-342), the filters ``chebyshev5`` / ``chebyshev2``
(same basis, lib/graph_conv.py:113-176) and ``fourier`` (:83-111), the
activations ``b1relu`` / ``b1tanh`` / ``b2relu`` (:178-199), ``mpool1`` /
``apool1`` (:201-218), ``fc`` (:220-226), the residual stack that calls them
(:234-330) and the pooled multi-level cgcnn (lib/models.py:61-127 with the
per-level conv / pool / fc inference the notebooks drive, usage.ipynb).
Every op runs on the HIP kernels of libcheb_mi355.so.  Everything else of the
TF model class (sessions, feeds, summaries) is outside the hot path.
"""
from __future__ import annotations

import contextlib

import numpy as np
import torch

from . import graph as host_graph
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
        self._fourier_cache: dict[int, tuple] = {}
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

    def _get_variable(self, leaf, shape, init):
        name = "/".join(self._scope + [leaf])
        w = self.weights.get(name)
        if w is None:
            w = torch.nn.Parameter(init(torch.empty(tuple(shape), device=self.device)))
            self.weights[name] = w
            self.nets[name] = w
        elif tuple(w.shape) != tuple(shape):
            raise ValueError(f"variable {name} exists with shape {tuple(w.shape)}, asked {tuple(shape)}")
        return w

    def _weight_variable(self, shape, regularization=True):
        """tf.get_variable('weights', shape, truncated_normal(0, 0.1)) in the
        current scope (lib/graph_model.py:326-333)."""
        return self._get_variable("weights", shape, lambda t: truncated_normal_(t, 0.1, self._gen))

    def _bias_variable(self, shape, regularization=True):
        """tf.get_variable('bias', shape, constant_initializer(0.1)) in the
        current scope (lib/graph_model.py:335-342)."""
        return self._get_variable("bias", shape, lambda t: t.fill_(0.1))

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

    def chebyshev2(self, x, L, Fout, K):
        """lib/graph_conv.py:113-142: the same basis (graph.chebyshev through
        tf.py_func), layout and contraction as chebyshev5 -- one HIP path."""
        return self.chebyshev5(x, L, Fout, K)

    def fourier(self, x, L, Fout, K):
        """lib/graph_conv.py:101-111 + filter_in_fourier :83-99.  U comes from
        the dense EVD of L (graph.fourier, host, once per L); W is
        [M, Fout, Fin].  The two transforms run on the MFMA GEMM, the
        per-frequency mix on its own kernel."""
        N, M, Fin = (int(s) for s in x.shape)
        U = self._fourier_basis(L, x.device)
        W = self._weight_variable([M, Fout, Fin], regularization=False)
        return ops.fourier_conv(x, W, U)

    def _fourier_basis(self, L, device):
        hit = self._fourier_cache.get(id(L))
        if hit is None or hit[0] is not L:
            _, U = host_graph.fourier(L)
            hit = (L, torch.as_tensor(np.ascontiguousarray(U, dtype=np.float32), device=device))
            self._fourier_cache[id(L)] = hit
        return hit[1]

    def _filter_act(self, x, L, Fout, K, residual=None):
        """brelu(filter(x) [+ residual]) -- fused into the filter's y store when
        the bound filter / activation are chebyshev5 (or chebyshev2) / b1relu
        (the residual block's `x = filter(x)`, `x = x + x_identity`,
        `x = brelu(x)`, lib/graph_conv.py:256-262); otherwise separate calls."""
        fuse = (getattr(self.filter, "__func__", None) in (GraphConv.chebyshev5, GraphConv.chebyshev2)
                and getattr(self.brelu, "__func__", None) is GraphConv.b1relu)
        if not fuse:
            y = self.filter(x, L, Fout, K)
            if residual is not None:
                y = y + residual
            return self.brelu(y)
        N, M, Fin = (int(s) for s in x.shape)
        plan = plan_for(L, lmax=2, device=x.device.index or 0, path=self.path)
        W = self._weight_variable([Fin * K, Fout], regularization=False)
        return ops.cheb_conv(x, W, plan, int(K), residual=residual, act="relu")

    # -- activations / pooling / dense ---------------------------------------------
    def b1relu(self, x):
        """lib/graph_conv.py:178-187 (its bias is commented out -> plain ReLU)."""
        return ops.bias_act(x, None, "relu")

    def b1tanh(self, x):
        """lib/graph_conv.py:189-193: tanh(x + b), one bias per filter [1, 1, F]."""
        b = self._bias_variable([1, 1, int(x.shape[-1])], regularization=False)
        return ops.bias_act(x, b, "tanh")

    def b2relu(self, x):
        """lib/graph_conv.py:195-199: relu(x + b), one bias per vertex and filter [1, M, F]."""
        b = self._bias_variable([1, int(x.shape[1]), int(x.shape[2])], regularization=False)
        return ops.bias_act(x, b, "relu")

    def mpool1(self, x, p):
        return ops.mpool1(x, int(p))

    def apool1(self, x, p):
        return ops.apool1(x, int(p))

    def fc(self, x, Mout, relu=True):
        """lib/graph_conv.py:220-226: relu(x [N, Min] @ W [Min, Mout] + b) on the
        MFMA GEMM and the bias/activation kernel."""
        Min = int(x.shape[1])
        W = self._weight_variable([Min, int(Mout)], regularization=True)
        b = self._bias_variable([int(Mout)], regularization=True)
        return ops.bias_act(ops.matmul(x, W), b, "relu" if relu else "none")

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

    def inference(self, x, L, nfilter, K, nres_layer_count, stack_num=1, groups=((0, 12), (12, 16)),
                  Fout_last=2):
        """``_inference`` (lib/graph_conv.py:272-303).  stack_num == 1: the
        residual network on x.  stack_num > 1: channel group i of x (the
        reference hard-codes [0:12] and [12:16], :284-285) through its own
        residual network in scope final_merge/VC_i, ReLU, merged as
        X = sum_i relu(net_i) * w_i with w_i = final_merge/W_i/weights [M, Fout_last]."""
        if stack_num == 1:
            return self.residual_network(x, L, nfilter, K, nres_layer_count, Fout_last)
        if len(groups) != stack_num:
            raise ValueError(f"stack_num={stack_num} needs {stack_num} channel groups, got {len(groups)}")
        C = int(x.shape[-1])
        X = None
        with self.variable_scope("final_merge"):
            for i, (a, b) in enumerate(groups):
                xi = x if (a, b) == (0, C) else ops.slice_channels(x, a, b)
                with self.variable_scope(f"VC_{i}"):
                    x1 = self.residual_network(xi, L, nfilter, K, nres_layer_count, Fout_last)
                with self.variable_scope(f"W_{i}"):
                    w1 = self._weight_variable([int(x1.shape[1]), int(x1.shape[2])])
                X = ops.stack_merge(x1, w1, X)
        return X

    # -- the pooled multi-level cgcnn (lib/models.py:61-127, usage.ipynb) ------------
    @staticmethod
    def select_laplacians(L, p):
        """lib/models.py:72-85: the Laplacian of each conv layer -- level j
        advances by log2(p_i) after layer i (p powers of 2)."""
        p_log2 = [int(np.log2(pp)) if pp > 1 else 0 for pp in p]
        if any(pp < 1 or (pp > 1 and 2 ** lg != pp) for pp, lg in zip(p, p_log2)):
            raise ValueError(f"pooling sizes must be powers of 2, got {list(p)}")
        if len(L) < 1 + sum(p_log2):
            raise ValueError(f"{len(L)} graph levels are too few for pooling sizes {list(p)}")
        out, j = [], 0
        for pp, lg in zip(p, p_log2):
            out.append(L[j])
            j += lg
        return out

    def cgcnn_inference(self, x, L, F, K, p, M):
        """conv{i}: pool(brelu(filter(x, L_i, F_i, K_i)), p_i) per graph level,
        then fc{i} (ReLU) layers and the linear ``logits`` layer.  Dropout is
        the identity here (inference; the reference's keep-probability 1 of
        usage.ipynb).  x: [N, M0] (one feature) or [N, M0, Fin], already in the
        coarsening order (perm_data)."""
        if not (len(F) == len(K) == len(p)) or len(L) < len(F):
            raise ValueError("need len(L) >= len(F) == len(K) == len(p) (lib/models.py:72)")
        Ls = self.select_laplacians(L, p)
        if x.dim() == 2:
            x = x.unsqueeze(2)
        for i in range(len(p)):
            with self.variable_scope(f"conv{i + 1}"):
                x = self._filter_act(x, Ls[i], int(F[i]), int(K[i]))
                x = self.pool(x, int(p[i]))
        x = x.reshape(int(x.shape[0]), -1)
        for i, Mi in enumerate(M[:-1]):
            with self.variable_scope(f"fc{i + 1}"):
                x = self.fc(x, int(Mi))
        with self.variable_scope("logits"):
            x = self.fc(x, int(M[-1]), relu=False)
        return x
