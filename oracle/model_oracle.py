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


# ---- stacked-input ResGNN: _inference with stack_num > 1 (lib/graph_conv.py:272-303)
def stacked_forward(x, nets, merge_Ws, groups, lap, K, R):
    """x [N, M, C]; nets[i] = Ws of network i (forward()'s layout), merge_Ws[i]
    [M, F].  X = sum_i relu(net_i(x[..., a_i:b_i])) * w_i (:284-301).
    Returns (X, caches)."""
    X = None
    caches = []
    for (a, b), Ws, w in zip(groups, nets, merge_Ws):
        out, cache = forward(np.asarray(x, np.float64)[..., a:b], Ws, lap, K, R)
        x1 = np.maximum(out, 0)                                   # (:292)
        X = x1 * w if X is None else X + x1 * w                   # (:297-301)
        caches.append((out, cache))
    return X, caches


def stacked_backward(dX, caches, nets, merge_Ws, lap, K, R):
    """Returns (dWs per network, dw per merge weight)."""
    dnets, dws = [], []
    for (out, cache), Ws, w in zip(caches, nets, merge_Ws):
        x1 = np.maximum(out, 0)
        dws.append(np.sum(dX * x1, axis=0))                       # Mul grad, reduced over N
        dout = dX * w * (out > 0)                                  # Mul grad, then ReluGrad
        dnets.append(backward(dout, cache, Ws, lap, K, R))
    return dnets, dws


def ema_update(state, value, decay=0.9):
    """tf.train.ExponentialMovingAverage(decay).apply([loss]) of a Tensor
    (lib/graph_model.py:265-273): zero-debiased assign_moving_average.
    state = (biased, average, local_step); returns the new state."""
    biased, avg, step = state
    d1 = 1.0 - decay
    biased = biased - (biased - value) * d1
    step = step + 1
    avg = avg - (avg - biased / (1.0 - (1.0 - d1) ** step))
    return biased, avg, step


def stacked_train_step(x, labels, nets, merge_Ws, groups, lap, K, R, adam_state, step, lr):
    """One step; adam_state in the order net_0 weights, w_0, net_1 weights, w_1, ...
    Returns (loss, grads in that order, new nets, new merge_Ws, new adam_state)."""
    X, caches = stacked_forward(x, nets, merge_Ws, groups, lap, K, R)
    loss, dX = loss_and_grad(X, labels)
    dnets, dws = stacked_backward(dX, caches, nets, merge_Ws, lap, K, R)
    flat_W, flat_g = [], []
    for Ws, w, gs, gw in zip(nets, merge_Ws, dnets, dws):
        flat_W += list(Ws) + [w]
        flat_g += list(gs) + [gw]
    new_flat, new_state = [], []
    for W, g, (m, v) in zip(flat_W, flat_g, adam_state):
        W2, m2, v2 = O.adam_step(W, g, m, v, step, lr=lr)
        new_flat.append(W2)
        new_state.append((m2, v2))
    new_nets, new_merge, i = [], [], 0
    for Ws in nets:
        new_nets.append(new_flat[i:i + len(Ws)])
        new_merge.append(new_flat[i + len(Ws)])
        i += len(Ws) + 1
    return loss, flat_g, new_nets, new_merge, new_state
