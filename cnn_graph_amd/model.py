"""The reference's ResGNN training step on device: ``GraphConv.residual_network``
(lib/graph_conv.py:234-330, ``model_name == 'ResGNN'``) + MSE loss
(lib/graph_model.py:246-275) + Adam with staircase exponential decay
(lib/graph_model.py:277-310), as ONE explicit schedule of C-ABI launches:

  conv_init    a   = relu(cheb(x; W_init))                       cg_cheb_forward_ex
  layer i      t   = relu(cheb(h; W_i0))                          (ReLU in the y store)
               h'  = relu(cheb(t; W_i1) + h)                      (residual + ReLU in the y store)
  convN        out = cheb(h; W_N)
  loss         mean((labels - out)^2), dout = 2 (out - labels) / n      cg_mse_loss
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
"""
from __future__ import annotations

import ctypes
import math

import torch

from . import _lib
from . import ops
from .graph_conv import truncated_normal_
from .plan import plan_for


class ResGNN:
    """ResGNN on one graph level (the fork's active model uses ``L[0]`` everywhere)."""

    def __init__(self, L, N: int, Fin: int, nfilter: int, K: int, nres_layer_count: int,
                 Fout_last: int = 2, learning_rate: float = 1e-3, decay_rate: float = 0.95,
                 decay_steps: int | None = None, device=None, seed: int = 2017, comm=None,
                 lmax: float = 2):
        self.device = torch.device(device if device is not None else "cuda")
        dev_index = self.device.index if self.device.index is not None else 0
        self.plan = plan_for(L, lmax=lmax, device=dev_index)
        self.M = M = self.plan.M
        self.N, self.Fin, self.nfilter, self.K = int(N), int(Fin), int(nfilter), int(K)
        self.R = int(nres_layer_count)
        self.lr, self.decay_rate, self.decay_steps = learning_rate, decay_rate, decay_steps
        self.comm = comm
        # (scope, Fin, Fout, act, residual-of) in the reference's call order
        layers = [("conv_init/weights", Fin, nfilter, "relu")]
        for i in range(self.R):
            layers.append((f"residual_layer_{i}/sublayer0/weights", nfilter, nfilter, "relu"))
            layers.append((f"residual_layer_{i}/sublayer1/weights", nfilter, nfilter, "relu"))
        layers.append(("convN/weights", nfilter, Fout_last, "none"))
        self.layers = layers
        f32 = dict(device=self.device, dtype=torch.float32)
        sizes = [fi * K * fo for _, fi, fo, _ in layers]
        total = sum(sizes)
        self.flat = torch.empty(total, **f32)
        self.grad = torch.zeros(total, **f32)
        self.m = torch.zeros(total, **f32)
        self.v = torch.zeros(total, **f32)
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed)
        self.W, self.dW, off = [], [], 0
        for (name, fi, fo, _), sz in zip(layers, sizes):
            w = self.flat[off:off + sz].view(fi * K, fo)
            truncated_normal_(w, 0.1, gen)
            self.W.append(w)
            self.dW.append(self.grad[off:off + sz].view(fi * K, fo))
            off += sz
        self.names = [name for name, *_ in layers]
        # activations / bases saved by the forward, gradient work buffers
        self.basis = [torch.empty((N * M, fi * K), **f32) for _, fi, _, _ in layers]
        self.out = [torch.empty((N, M, fo), **f32) for _, _, fo, _ in layers]
        self.g_a = torch.empty((N, M, nfilter), **f32)
        self.g_b = torch.empty((N, M, nfilter), **f32)
        self.g_c = torch.empty((N, M, nfilter), **f32)
        self.loss = torch.empty((1,), **f32)
        self.dout = torch.empty((N, M, Fout_last), **f32)
        self.step_count = 0
        fb = max(self.plan.workspace_bytes(N, fi, K, fo)[0] for _, fi, fo, _ in layers)
        bb = max(self.plan.workspace_bytes(N, fi, K, fo)[1] for _, fi, fo, _ in layers)
        # one workspace serves every forward and backward call (stream order:
        # a call's workspace is dead once the call has executed)
        self.fws = self.bws = torch.empty(max(fb, bb, 1), device=self.device, dtype=torch.uint8)
        self.fws_n, self.bws_n = fb, bb
        nb = ctypes.c_size_t()
        _lib.call("cg_mse_loss_workspace_bytes", N * M * Fout_last, ctypes.byref(nb))
        self.mws = torch.empty(max(nb.value, 1), device=self.device, dtype=torch.uint8)
        self.mws_n = nb.value
        h = _lib.lib()
        self._fwd, self._bwd, self._mse, self._adam = (h.cg_cheb_forward_ex, h.cg_cheb_backward_ex,
                                                       h.cg_mse_loss, h.cg_adam_update)

    def parameters(self):
        return dict(zip(self.names, self.W))

    def gradients(self):
        return dict(zip(self.names, self.dW))

    # -- schedule pieces ------------------------------------------------------------
    def _f(self, li, x, res, s):
        _, fi, fo, act = self.layers[li]
        st = self._fwd(self.plan.handle, self.N, fi, self.K, fo, x.data_ptr(), self.W[li].data_ptr(),
                       res.data_ptr() if res is not None else None, ops.ACTS[act],
                       self.basis[li].data_ptr(), self.out[li].data_ptr(), self.fws.data_ptr(),
                       self.fws_n, s)
        _lib.check("cg_cheb_forward_ex", st)
        return self.out[li]

    def _b(self, li, dy, dz, dx, dx_acc, s):
        _, fi, fo, act = self.layers[li]
        st = self._bwd(self.plan.handle, self.N, fi, self.K, fo, dy.data_ptr(),
                       self.out[li].data_ptr(), ops.ACTS[act], self.basis[li].data_ptr(),
                       self.W[li].data_ptr(), dx.data_ptr() if dx is not None else None,
                       int(dx_acc), self.dW[li].data_ptr(), dz.data_ptr() if dz is not None else None,
                       self.bws.data_ptr(), self.bws_n, s)
        _lib.check("cg_cheb_backward_ex", st)

    def forward(self, x, stream=None):
        """residual_network (lib/graph_conv.py:305-330): returns the logits [N, M, Fout_last]."""
        s = stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream
        if tuple(x.shape) != (self.N, self.M, self.Fin) or not x.is_cuda:
            raise ValueError(f"x must be a cuda tensor of shape {(self.N, self.M, self.Fin)}")
        x = x.contiguous()
        h = self._f(0, x, None, s)
        li = 1
        for _ in range(self.R):
            t = self._f(li, h, None, s)
            h = self._f(li + 1, t, h, s)
            li += 2
        return self._f(li, h, None, s)

    def learning_rate(self, step):
        """tf.train.exponential_decay(lr, global_step, decay_steps, decay_rate, staircase=True)."""
        if self.decay_rate == 1 or not self.decay_steps:
            return self.lr
        return self.lr * self.decay_rate ** math.floor(step / self.decay_steps)

    def train_step(self, x, labels, stream=None):
        """One optimizer step (lib/graph_model.py:277-310); returns the device loss [1]."""
        s = stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream
        out = self.forward(x, s)
        n = out.numel()
        labels = labels.contiguous()
        if labels.numel() != n:
            raise ValueError("labels must match the logits' shape")
        _lib.check("cg_mse_loss", self._mse(out.data_ptr(), labels.data_ptr(), n,
                                            self.loss.data_ptr(), self.dout.data_ptr(),
                                            self.mws.data_ptr(), self.mws_n, s))
        last = len(self.layers) - 1
        dh = self.g_a
        self._b(last, self.dout, None, dh, False, s)           # convN: dh = dL/dh
        bufs = [self.g_a, self.g_b, self.g_c]
        cur = 0  # bufs[cur] is dh
        li = last - 2
        for _ in range(self.R):
            dz1 = bufs[(cur + 1) % 3]
            dt = bufs[(cur + 2) % 3]
            self._b(li + 1, dh, dz1, dt, False, s)             # sublayer1: dz1 = dh*[h'>0] (= d residual)
            self._b(li, dt, dh, dz1, True, s)                  # sublayer0: dz1 += dx  (dh buffer as dz0)
            dh, cur = dz1, (cur + 1) % 3
            li -= 2
        self._b(0, dh, bufs[(cur + 1) % 3], None, False, s)     # conv_init (no dx: x is data)
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
        return self.loss
