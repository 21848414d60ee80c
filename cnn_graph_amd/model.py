"""The reference's ResGNN training step on device: ``GraphConv.residual_network``
(lib/graph_conv.py:234-330, ``model_name == 'ResGNN'``) + MSE loss
(lib/graph_model.py:246-275) + Adam with staircase exponential decay
(lib/graph_model.py:277-310), as ONE explicit schedule of C-ABI launches:

  conv_init    a   = relu(cheb(x; W_init))                       cg_cheb_forward_ex
  layer i      t   = relu(cheb(h; W_i0))                          (ReLU in the y store)
               h'  = relu(cheb(t; W_i1) + h)                      (residual + ReLU in the y store)
  convN        out = cheb(h; W_N)
  loss         mean((labels - out)^2), dout = 2 (out - labels) / n, and the
               loss moving average (lib/graph_model.py:265-273)    cg_mse_loss_ema
  (filters whose forward and backward both run the sample-major streaming
  path with Fin % 16 == 0 -- the hidden layers at the humanflow shape -- keep
  their basis in the planes layout, cg_cheb_forward_layout(CG_BASIS_PLANES):
  each Chebyshev step writes its own plane, no rows-layout assembly pass)
  backward     cg_cheb_backward_ex per filter in reverse: ReLU mask from the
               saved outputs, the residual branch's gradient dz1 doubles as the
               buffer the sublayer-0 input gradient is ACCUMULATED into
               (dx_accumulate), so dh_in = dx(f0) + dz1 needs no extra pass
  exchange     one all-reduce of the flat gradient buffer (RcclComm, N > 1)
  update       ONE cg_adam_update over the flat parameter buffer (grad / world)

Every weight is a view into one flat fp32 buffer (and so is every gradient),
so the optimizer and the data-parallel exchange are one launch each.  No
PyTorch compute op runs in the step: torch only owns the buffers.
Weights: ``truncated_normal(0, 0.1)`` per ``tf.get_variable('weights')``
(lib/graph_model.py:326-333) in the reference's scope order.

``StackedResGNN`` is ``_inference`` with ``stack_num > 1`` (lib/graph_conv.py:
272-303, the ``_STACK_NUM = 2`` driver nips2016/humanflow-ln-period-shortlong.py
:171): the input's channel groups (``x[..., 0:12]`` and ``x[..., 12:16]``) run
through separate residual networks, merged as ``X = sum_i relu(net_i) * w_i``
with ``w_i [M, 2]`` -- same flat-buffer schedule, one Adam, one all-reduce.
"""
from __future__ import annotations

import ctypes
import math

import torch

from . import _lib
from . import ops
from .graph_conv import truncated_normal_
from .plan import plan_for


class _ResNet:
    """One ``residual_network`` (lib/graph_conv.py:305-330): conv_init, R
    residual layers of two filters each, convN.  Its weights and gradients are
    views into the owner's flat buffers starting at ``off``."""

    def __init__(self, owner, scope: str, Fin: int, off: int, gen):
        self.o = owner
        N, M, K, F = owner.N, owner.M, owner.K, owner.nfilter
        # (scope, Fin, Fout, act) in the reference's call order
        layers = [(f"{scope}conv_init/weights", Fin, F, "relu")]
        for i in range(owner.R):
            layers.append((f"{scope}residual_layer_{i}/sublayer0/weights", F, F, "relu"))
            layers.append((f"{scope}residual_layer_{i}/sublayer1/weights", F, F, "relu"))
        layers.append((f"{scope}convN/weights", F, owner.Fout_last, "none"))
        self.layers = layers
        self.Fin = Fin
        f32 = dict(device=owner.device, dtype=torch.float32)
        self.W, self.dW = [], []
        for _, fi, fo, _ in layers:
            sz = fi * K * fo
            w = owner.flat[off:off + sz].view(fi * K, fo)
            truncated_normal_(w, 0.1, gen)
            self.W.append(w)
            self.dW.append(owner.grad[off:off + sz].view(fi * K, fo))
            off += sz
        self.end = off
        self.names = [name for name, *_ in layers]
        # activations / bases saved by the forward, gradient work buffers; the
        # basis layout per filter: planes where it applies, else rows
        self.layout = ["planes" if owner.plan.basis_elems(N, fi, K, fo, "planes") else "rows"
                       for _, fi, fo, _ in layers]
        self.basis = [torch.empty((K, N * M, fi) if lay == "planes" else (N * M, fi * K), **f32)
                      for (_, fi, _, _), lay in zip(layers, self.layout)]
        self.out = [torch.empty((N, M, fo), **f32) for _, _, fo, _ in layers]
        self.g = [torch.empty((N, M, F), **f32) for _ in range(3)]

    @staticmethod
    def sizes(Fin, F, K, R, Fout_last):
        return [Fin * K * F] + [F * K * F] * (2 * R) + [F * K * Fout_last]

    def ws_bytes(self):
        o = self.o
        fb = max(o.plan.workspace_bytes(o.N, fi, o.K, fo)[0] for _, fi, fo, _ in self.layers)
        bb = max(o.plan.workspace_bytes(o.N, fi, o.K, fo)[1] for _, fi, fo, _ in self.layers)
        return max(fb, bb)

    def _f(self, li, x, res, s):
        o = self.o
        _, fi, fo, act = self.layers[li]
        st = o._fwd(o.plan.handle, o.N, fi, o.K, fo, x.data_ptr(), self.W[li].data_ptr(),
                    res.data_ptr() if res is not None else None, ops.ACTS[act],
                    _lib.BASIS_LAYOUTS[self.layout[li]], self.basis[li].data_ptr(),
                    self.out[li].data_ptr(), o.ws.data_ptr(), o.ws_n, s)
        _lib.check("cg_cheb_forward_layout", st)
        return self.out[li]

    def _b(self, li, dy, dz, dx, dx_acc, s):
        o = self.o
        _, fi, fo, act = self.layers[li]
        st = o._bwd(o.plan.handle, o.N, fi, o.K, fo, dy.data_ptr(), self.out[li].data_ptr(),
                    ops.ACTS[act], _lib.BASIS_LAYOUTS[self.layout[li]], self.basis[li].data_ptr(),
                    self.W[li].data_ptr(), dx.data_ptr() if dx is not None else None, int(dx_acc),
                    self.dW[li].data_ptr(), dz.data_ptr() if dz is not None else None,
                    o.ws.data_ptr(), o.ws_n, s)
        _lib.check("cg_cheb_backward_layout", st)

    def forward(self, x, s):
        h = self._f(0, x, None, s)
        li = 1
        for _ in range(self.o.R):
            t = self._f(li, h, None, s)
            h = self._f(li + 1, t, h, s)
            li += 2
        return self._f(li, h, None, s)

    def backward(self, dout, s):
        """Every dW of this network from d(out); the input gets no gradient (data)."""
        last = len(self.layers) - 1
        bufs = self.g
        dh = bufs[0]
        self._b(last, dout, None, dh, False, s)            # convN: dh = dL/dh
        cur = 0  # bufs[cur] is dh
        li = last - 2
        for _ in range(self.o.R):
            dz1 = bufs[(cur + 1) % 3]
            dt = bufs[(cur + 2) % 3]
            self._b(li + 1, dh, dz1, dt, False, s)         # sublayer1: dz1 = dh*[h'>0] (= d residual)
            self._b(li, dt, dh, dz1, True, s)              # sublayer0: dz1 += dx  (dh buffer as dz0)
            dh, cur = dz1, (cur + 1) % 3
            li -= 2
        self._b(0, dh, bufs[(cur + 1) % 3], None, False, s)  # conv_init (no dx: x is data)


class _Trainer:
    """Shared pieces of the explicit training schedules: flat parameter /
    gradient / Adam buffers, the MSE loss with its moving average, the
    exchange and the one Adam launch (lib/graph_model.py:246-310)."""

    def _setup(self, L, N, nfilter, K, nres_layer_count, Fout_last, learning_rate, decay_rate,
               decay_steps, device, comm, lmax, total):
        self.device = torch.device(device if device is not None else "cuda")
        dev_index = self.device.index if self.device.index is not None else 0
        self.plan = plan_for(L, lmax=lmax, device=dev_index)
        self.M = self.plan.M
        self.N, self.nfilter, self.K = int(N), int(nfilter), int(K)
        self.R, self.Fout_last = int(nres_layer_count), int(Fout_last)
        self.lr, self.decay_rate, self.decay_steps = learning_rate, decay_rate, decay_steps
        self.comm = comm
        f32 = dict(device=self.device, dtype=torch.float32)
        self.flat = torch.empty(total, **f32)
        self.grad = torch.zeros(total, **f32)
        self.m = torch.zeros(total, **f32)
        self.v = torch.zeros(total, **f32)
        self.loss = torch.empty((1,), **f32)
        # {biased, average, local_step} of ExponentialMovingAverage(0.9) of the loss
        self.ema = torch.zeros((3,), **f32)
        self.dout = torch.empty((self.N, self.M, self.Fout_last), **f32)
        self.step_count = 0
        nb = ctypes.c_size_t()
        _lib.call("cg_mse_loss_workspace_bytes", self.N * self.M * self.Fout_last, ctypes.byref(nb))
        self.mws = torch.empty(max(nb.value, 1), device=self.device, dtype=torch.uint8)
        self.mws_n = nb.value
        h = _lib.lib()
        self._fwd, self._bwd, self._mse, self._adam = (h.cg_cheb_forward_layout,
                                                       h.cg_cheb_backward_layout,
                                                       h.cg_mse_loss_ema, h.cg_adam_update)

    def _alloc_ws(self, nets):
        # one workspace serves every forward and backward call (stream order:
        # a call's workspace is dead once the call has executed)
        self.ws_n = max(n.ws_bytes() for n in nets)
        self.ws = torch.empty(max(self.ws_n, 1), device=self.device, dtype=torch.uint8)

    @property
    def loss_average(self):
        """The loss moving average (lib/graph_model.py:271-273), a device scalar."""
        return self.ema[1:2]

    def learning_rate(self, step):
        """tf.train.exponential_decay(lr, global_step, decay_steps, decay_rate, staircase=True)."""
        if self.decay_rate == 1 or not self.decay_steps:
            return self.lr
        return self.lr * self.decay_rate ** math.floor(step / self.decay_steps)

    def _loss(self, out, labels, s):
        n = out.numel()
        labels = labels.contiguous()
        if labels.numel() != n:
            raise ValueError("labels must match the logits' shape")
        _lib.check("cg_mse_loss_ema", self._mse(out.data_ptr(), labels.data_ptr(), n,
                                                self.loss.data_ptr(), self.dout.data_ptr(),
                                                self.ema.data_ptr(), ctypes.c_float(0.9),
                                                self.mws.data_ptr(), self.mws_n, s))

    def _exchange_and_update(self, s):
        world = 1
        if self.comm is not None and self.comm.world > 1:
            self.comm.allreduce_sum_(self.grad, s)
            world = self.comm.world
        self.step_count += 1
        lr = self.learning_rate(self.step_count - 1)
        _lib.check("cg_adam_update", self._adam(
            self.flat.data_ptr(), self.grad.data_ptr(), self.m.data_ptr(), self.v.data_ptr(),
            self.flat.numel(), ctypes.c_float(lr), ctypes.c_float(0.9), ctypes.c_float(0.999),
            ctypes.c_float(1e-8), self.step_count, ctypes.c_float(1.0 / world), s))

    def _stream(self, stream):
        return stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream

    def parameters(self):
        return dict(zip(self.names, self.W))

    def gradients(self):
        return dict(zip(self.names, self.dW))


class ResGNN(_Trainer):
    """ResGNN on one graph level (the fork's active model uses ``L[0]`` everywhere)."""

    def __init__(self, L, N: int, Fin: int, nfilter: int, K: int, nres_layer_count: int,
                 Fout_last: int = 2, learning_rate: float = 1e-3, decay_rate: float = 0.95,
                 decay_steps: int | None = None, device=None, seed: int = 2017, comm=None,
                 lmax: float = 2):
        total = sum(_ResNet.sizes(Fin, nfilter, K, nres_layer_count, Fout_last))
        self._setup(L, N, nfilter, K, nres_layer_count, Fout_last, learning_rate, decay_rate,
                    decay_steps, device, comm, lmax, total)
        self.Fin = int(Fin)
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed)
        self.net = _ResNet(self, "", self.Fin, 0, gen)
        self.layers, self.names = self.net.layers, self.net.names
        self.W, self.dW = self.net.W, self.net.dW
        self.basis, self.out = self.net.basis, self.net.out
        self._alloc_ws([self.net])

    def forward(self, x, stream=None):
        """residual_network (lib/graph_conv.py:305-330): returns the logits [N, M, Fout_last]."""
        s = self._stream(stream)
        if tuple(x.shape) != (self.N, self.M, self.Fin) or not x.is_cuda:
            raise ValueError(f"x must be a cuda tensor of shape {(self.N, self.M, self.Fin)}")
        return self.net.forward(x.contiguous(), s)

    def train_step(self, x, labels, stream=None):
        """One optimizer step (lib/graph_model.py:277-310); returns the device loss [1]."""
        s = self._stream(stream)
        out = self.forward(x, s)
        self._loss(out, labels, s)
        self.net.backward(self.dout, s)
        self._exchange_and_update(s)
        return self.loss


class StackedResGNN(_Trainer):
    """``GraphConv._inference`` with ``stack_num > 1`` (lib/graph_conv.py:272-303).

    ``groups`` are the channel ranges of the input fed to each residual
    network; the reference hard-codes ``x_arr[0:12]`` and ``x_arr[12:16]``
    (:284-285) for its 16-channel (8 periods x 2 flows) humanflow input.
    Variable order (= initialisation order): for each i, the network
    ``final_merge/VC_i/...`` then the merge weight ``final_merge/W_i/weights``
    [M, Fout_last]."""

    def __init__(self, L, N: int, C: int, nfilter: int, K: int, nres_layer_count: int,
                 groups=((0, 12), (12, 16)), Fout_last: int = 2, learning_rate: float = 1e-3,
                 decay_rate: float = 0.95, decay_steps: int | None = None, device=None,
                 seed: int = 2017, comm=None, lmax: float = 2):
        groups = [(int(a), int(b)) for a, b in groups]
        if len(groups) < 1 or any(not (0 <= a < b <= C) for a, b in groups):
            raise ValueError(f"bad channel groups {groups} for C={C}")
        self.C, self.groups = int(C), groups
        M = L.shape[0]
        sizes = [sum(_ResNet.sizes(b - a, nfilter, K, nres_layer_count, Fout_last)) + M * Fout_last
                 for a, b in groups]
        self._setup(L, N, nfilter, K, nres_layer_count, Fout_last, learning_rate, decay_rate,
                    decay_steps, device, comm, lmax, sum(sizes))
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed)
        f32 = dict(device=self.device, dtype=torch.float32)
        self.nets, self.merge_W, self.merge_dW = [], [], []
        self.W, self.dW, self.names = [], [], []
        off = 0
        for i, (a, b) in enumerate(groups):
            net = _ResNet(self, f"final_merge/VC_{i}/", b - a, off, gen)
            off = net.end
            mf = self.M * self.Fout_last
            w = self.flat[off:off + mf].view(self.M, self.Fout_last)
            truncated_normal_(w, 0.1, gen)
            dw = self.grad[off:off + mf].view(self.M, self.Fout_last)
            off += mf
            self.nets.append(net)
            self.merge_W.append(w)
            self.merge_dW.append(dw)
            self.W += net.W + [w]
            self.dW += net.dW + [dw]
            self.names += net.names + [f"final_merge/W_{i}/weights"]
        self.x_groups = [torch.empty((self.N, self.M, b - a), **f32) if (a, b) != (0, self.C) else None
                         for a, b in groups]
        self.X = torch.empty((self.N, self.M, self.Fout_last), **f32)
        self.d_net = torch.empty((self.N, self.M, self.Fout_last), **f32)
        self._alloc_ws(self.nets)
        h = _lib.lib()
        self._slice, self._merge_f, self._merge_b = (h.cg_slice_channels, h.cg_stack_merge_forward,
                                                     h.cg_stack_merge_backward)

    def forward(self, x, stream=None):
        """_inference (lib/graph_conv.py:274-303): returns X [N, M, Fout_last]."""
        s = self._stream(stream)
        if tuple(x.shape) != (self.N, self.M, self.C) or not x.is_cuda:
            raise ValueError(f"x must be a cuda tensor of shape {(self.N, self.M, self.C)}")
        x = x.contiguous()
        N, M, F = self.N, self.M, self.Fout_last
        for i, ((a, b), net) in enumerate(zip(self.groups, self.nets)):
            xi = x
            if self.x_groups[i] is not None:
                xi = self.x_groups[i]
                _lib.check("cg_slice_channels",
                           self._slice(x.data_ptr(), N * M, self.C, a, b, xi.data_ptr(), s))
            out = net.forward(xi, s)
            _lib.check("cg_stack_merge_forward",
                       self._merge_f(N, M, F, out.data_ptr(), self.merge_W[i].data_ptr(), int(i > 0),
                                     self.X.data_ptr(), s))
        return self.X

    def train_step(self, x, labels, stream=None):
        """One optimizer step over every network and merge weight; returns the device loss [1]."""
        s = self._stream(stream)
        X = self.forward(x, s)
        self._loss(X, labels, s)
        N, M, F = self.N, self.M, self.Fout_last
        for i, net in enumerate(self.nets):
            out = net.out[-1]
            _lib.check("cg_stack_merge_backward",
                       self._merge_b(N, M, F, self.dout.data_ptr(), out.data_ptr(),
                                     self.merge_W[i].data_ptr(), self.d_net.data_ptr(),
                                     self.merge_dW[i].data_ptr(), s))
            net.backward(self.d_net, s)
        self._exchange_and_update(s)
        return self.loss
