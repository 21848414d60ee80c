"""The data-parallel chebyshev5 training step that bench.py times, as an object
the tests can drive at any world size (lib/graph_model.py:277-298: the
exchange sits between compute_gradients and apply_gradients).

One step = forward (basis + y = basis W), backward (dx, dW against a fixed
upstream dy), the gradient exchange (sum over ranks) when there is one, and the
TF-1.x Adam update of W with the gradient scaled by 1/world.  Where the update
runs depends on the schedule:

  "fused"    (no exchange, one GPU) the update rides on the dW slab reduction:
             cg_cheb_backward_adam, no separate launch
  "forward"  (exchange) step i's forward applies step i-1's exchanged gradient
             in its prologue (cg_cheb_forward_adam): W, m and v double-buffered,
             so every step is forward + backward + all-reduce and nothing else;
             ``finish`` applies the last step's update
  "unfused"  cg_adam_update after the exchange (the ablation)

Every schedule applies the same updates in the same order: after ``finish``
the weights equal n forward/backward/exchange/Adam steps of the unfused loop
(bitwise: the fused forms reuse k_adam's expressions, tests/test_gpu_fused_adam.py
and tests/test_gpu_dp_bench.py).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib


class ChebTrainStep:
    """The schedule over a pre-allocated ``ops.ChebRunner``.

    allreduce: None (no exchange) or a callable ``allreduce(stream)`` that sums
    ``runner.dW`` over the ranks in place, enqueued on ``stream`` (bench.py
    passes the pre-bound cg_allreduce_sum_f32 call; tests pass a
    dist.TorchComm over gloo)."""

    def __init__(self, runner, x, dy, W, world: int = 1, allreduce=None, schedule: str = "auto",
                 lr: float = 1e-3, beta1: float = 0.9, beta2: float = 0.999, eps: float = 1e-8,
                 grad_scale: float | None = None):
        if schedule == "auto":
            schedule = "forward" if allreduce is not None else "fused"
        if schedule not in ("fused", "forward", "unfused"):
            raise ValueError(f"unknown schedule {schedule!r}")
        if schedule == "fused" and allreduce is not None:
            raise ValueError("the fused schedule has no exchange step (Adam runs inside the "
                             "dW reduction, before an all-reduce could)")
        self.runner, self.x, self.dy = runner, x, dy
        self.world, self.allreduce, self.schedule = int(world), allreduce, schedule
        self.hp = (float(lr), float(beta1), float(beta2), float(eps))
        # the loss is a batch mean (lib/graph_model.py:255): the exchanged sum / world
        self.scale = 1.0 / self.world if grad_scale is None else float(grad_scale)
        self.W = [W, torch.empty_like(W)]
        self.m = [torch.zeros_like(W), torch.zeros_like(W)]
        self.v = [torch.zeros_like(W), torch.zeros_like(W)]
        self._adam = _lib.lib().cg_adam_update
        self._adam_hp = tuple(ctypes.c_float(h) for h in self.hp)

    def _adam_update(self, W, m, v, step: int, stream):
        lr, b1, b2, eps = self._adam_hp
        st = self._adam(W.data_ptr(), self.runner.dW.data_ptr(), m.data_ptr(), v.data_ptr(),
                        W.numel(), lr, b1, b2, eps, int(step), ctypes.c_float(self.scale), stream)
        if st:
            _lib.check("cg_adam_update", st)

    def step(self, i: int, stream):
        """Training step i (0-based): its forward sees the weights after i updates."""
        r, lr, b1, b2, eps = self.runner, *self.hp
        if self.schedule == "forward":
            if i == 0:
                r.forward(self.x, self.W[0], stream=stream)
            else:
                pi, ci = (i - 1) % 2, i % 2
                r.forward_adam(self.x, self.W[pi], r.dW, self.m[pi], self.v[pi], self.W[ci],
                               self.m[ci], self.v[ci], i, lr, b1, b2, eps,
                               grad_scale=self.scale, stream=stream)
            Wc = self.W[i % 2]
        else:
            Wc = self.W[0]
            r.forward(self.x, Wc, stream=stream)
        if self.schedule == "fused":
            r.backward_adam(self.dy, Wc, self.m[0], self.v[0], i + 1, lr, b1, b2, eps,
                            grad_scale=self.scale, stream=stream)
            return
        r.backward(self.dy, Wc, stream=stream)
        if self.allreduce is not None:
            self.allreduce(stream)
        if self.schedule == "unfused":
            self._adam_update(Wc, self.m[0], self.v[0], i + 1, stream)

    def finish(self, n: int, stream):
        """After steps 0..n-1: the weights after all n updates (the forward
        schedule's last update, pending for a next forward, is applied here)."""
        if self.schedule != "forward":
            return self.W[0]
        j = (n - 1) % 2
        self._adam_update(self.W[j], self.m[j], self.v[j], n, stream)
        return self.W[j]
