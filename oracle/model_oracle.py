"""CPU oracle for the ResGNN training step.

TEST INFRASTRUCTURE ONLY: imported by ``tests/`` as the checker, never by
``cnn_graph_amd/``.

float64 restatement of lib/graph_conv.py::residual_network / residual_layer
(:234-330, ``model_name == 'ResGNN'``, activation 'brelu' = b1relu = ReLU with
its bias commented out, :178-187), the MSE loss (lib/graph_model.py:255) and
its TF autodiff gradient, followed by TF-1.x Adam (cheb_oracle.adam_step).
Each filter is ``lstm_oracle.cheb_conv64`` (cheby_conv in float64) and
``cheb_oracle.cheb_backward``.  TF is not installed, so this is pinned only
through its pieces (the pinned Chebyshev oracle) and, in tests, by finite
differences of its loss.
"""
from __future__ import annotations

import numpy as np

from . import cheb_oracle as O
from .lstm_oracle import cheb_conv64


def forward(x, Ws, lap, K, R):
    """Ws: [W_init, (W_i0, W_i1) * R, W_N].  Returns (out, cache)."""
    cache = []
    h = np.asarray(x, np.float64)

    def f(inp, W, res, act):
        A, y = cheb_conv64(inp, lap, W, K)
        pre = y + res if res is not None else y
        out = np.maximum(pre, 0) if act else pre
        cache.append((inp, A, out, act))
        return out

    h = f(h, Ws[0], None, True)
    li = 1
    for _ in range(R):
        t = f(h, Ws[li], None, True)
        h = f(t, Ws[li + 1], h, True)
        li += 2
    out = f(h, Ws[li], None, False)
    return out, cache


def loss_and_grad(out, labels):
    """tf.reduce_mean(tf.square(labels - logits)) and d/d logits."""
    d = np.asarray(labels, np.float64) - out
    return float(np.mean(d * d)), -2.0 * d / d.size


def backward(dout, cache, Ws, lap, K, R):
    """Returns the list of dW in the order of Ws."""
    rowptr, col, val = lap
    dWs = [None] * len(Ws)

    def b(li, dy):
        inp, A, out, act = cache[li]
        dz = dy * (out > 0) if act else dy
        N, M, Fin = inp.shape
        dx, dW = O.cheb_backward(dz, A, Ws[li], rowptr, col, val, N, M, Fin, K)
        dWs[li] = dW
        return dx, dz

    last = len(Ws) - 1
    dh, _ = b(last, dout)
    li = last - 2
    for _ in range(R):
        dt, dz1 = b(li + 1, dh)
        dx0, _ = b(li, dt)
        dh = dx0 + dz1
        li -= 2
    b(0, dh)
    return dWs


def train_step(x, labels, Ws, lap, K, R, adam_state, step, lr):
    """One step: returns (loss, dWs, new Ws, new adam_state)."""
    out, cache = forward(x, Ws, lap, K, R)
    loss, dout = loss_and_grad(out, labels)
    dWs = backward(dout, cache, Ws, lap, K, R)
    new_W, new_state = [], []
    for W, g, (m, v) in zip(Ws, dWs, adam_state):
        W2, m2, v2 = O.adam_step(W, g, m, v, step, lr=lr)
        new_W.append(W2)
        new_state.append((m2, v2))
    return loss, dWs, new_W, new_state
