"""CPU oracle for the gconv-LSTM cell.

TEST INFRASTRUCTURE ONLY: imported by ``tests/`` as the checker, never by
``cnn_graph_amd/``.

A float64 NumPy restatement of ``lib/gconv_lstm.py::GConvLSTMCell.__call__``
(lib/gconv_lstm.py:77-221) driven by ``tf.nn.static_rnn`` over a
``MultiRNNCell`` (lib/gconv_lstm.py:609-627), and of its TF autodiff
gradient (backprop through time).  The eight ``cheby_conv`` calls of a cell
(lib/filter.py:45-95) are restated with ``cheb_oracle``'s basis / layout /
contraction in float64.

Parity: TensorFlow is not installed, so nothing pins this restatement to TF
outputs (TF boundary unpinned); its backward is pinned to its
own forward by central finite differences (tests/test_lstm_oracle.py), and
its Chebyshev pieces are the pinned ``cheb_oracle`` functions.
"""
from __future__ import annotations

import numpy as np

from . import cheb_oracle as O

GATES = ("z", "i", "f", "o")


def _sigmoid(a):
    return 1.0 / (1.0 + np.exp(-a))


def cheb_conv64(x, lap, W, K):
    """cheby_conv(x, L, lmax, Fout, K, W) (lib/filter.py:45-95) in float64:
    returns (basis [N*M, Fin*K], y [N, M, Fout]).  lap = (rowptr, col, val) of L~."""
    rowptr, col, val = lap
    N, M, Fin = x.shape
    X0 = O.input_layout(np.asarray(x, np.float64))
    Xt = O.chebyshev_basis(rowptr, col, np.asarray(val, np.float64), X0, K)
    A = O.basis_layout(Xt, N, M, Fin, K)
    return A, (A @ np.asarray(W, np.float64)).reshape(N, M, W.shape[1])


def cell_forward(x, c, h, Wx, Wh, b, lap, K, H, gates="reference"):
    """One GConvLSTMCell step (lib/gconv_lstm.py:183-221).

    Wx [K*Fin, 4H] = [Wzxt | Wixt | Wfxt | Woxt], Wh [K*H, 4H], b [4H] =
    [bzt | bit | bft | bot] -- the reference's per-gate variables
    (:98-115, :173-176) concatenated column-wise.  gates="reference" keeps the
    reference's z = tan (:188) and o = tanh (:209); "standard" uses tanh /
    sigmoid.  Returns (c', h', cache)."""
    N, M, _ = x.shape
    Ax, gx = cheb_conv64(x, lap, Wx, K)
    Ah, gh = cheb_conv64(h, lap, Wh, K)
    a = gx + gh + np.asarray(b, np.float64)                       # (:186-187 ...)
    az, ai, af, ao = (a[..., q * H:(q + 1) * H] for q in range(4))
    z = np.tan(az) if gates == "reference" else np.tanh(az)
    i, f = _sigmoid(ai), _sigmoid(af)
    o = np.tanh(ao) if gates == "reference" else _sigmoid(ao)
    c = np.asarray(c, np.float64)
    cn = f * c + i * z                                           # (:215)
    hn = o * np.tanh(cn)                                         # (:218)
    cache = dict(x=x, h=h, c=c, cn=cn, z=z, i=i, f=f, o=o, Ax=Ax, Ah=Ah, N=N, M=M)
    return cn, hn, cache


def cell_backward(dh, dc, cache, Wx, Wh, lap, K, H, gates="reference"):
    """Gradient of cell_forward: returns (dx, dc_prev, dh_prev, dWx, dWh, db, dpre)."""
    z, i, f, o, c, cn = (cache[k] for k in ("z", "i", "f", "o", "c", "cn"))
    N, M = cache["N"], cache["M"]
    rowptr, col, val = lap
    tc = np.tanh(cn)
    dcn = dh * o * (1 - tc * tc) + dc
    d_o = dh * tc
    d_z, d_i, d_f = dcn * i, dcn * z, dcn * c
    daz = d_z * (1 + z * z) if gates == "reference" else d_z * (1 - z * z)
    dai, daf = d_i * i * (1 - i), d_f * f * (1 - f)
    dao = d_o * (1 - o * o) if gates == "reference" else d_o * o * (1 - o)
    dpre = np.concatenate([daz, dai, daf, dao], axis=-1)         # [N, M, 4H]
    Fin = cache["x"].shape[2]
    dx, dWx = O.cheb_backward(dpre, cache["Ax"], Wx, rowptr, col, val, N, M, Fin, K)
    dh_prev, dWh = O.cheb_backward(dpre, cache["Ah"], Wh, rowptr, col, val, N, M, H, K)
    db = dpre.reshape(-1, 4 * H).sum(axis=0)
    return dx, dcn * f, dh_prev, dWx, dWh, db, dpre


def layer_forward(xs, params, lap, K, H, c0=None, h0=None, gates="reference"):
    """static_rnn of one cell over xs [T, N, M, Fin] from (c0, h0) (zero state
    of :71-76 when None).  Returns (hs [T, N, M, H], cs [T, N, M, H], caches)."""
    Wx, Wh, b = params
    T, N, M, _ = xs.shape
    c = np.zeros((N, M, H)) if c0 is None else np.asarray(c0, np.float64)
    h = np.zeros((N, M, H)) if h0 is None else np.asarray(h0, np.float64)
    hs, cs, caches = [], [], []
    for t in range(T):
        c, h, cache = cell_forward(xs[t], c, h, Wx, Wh, b, lap, K, H, gates)
        hs.append(h)
        cs.append(c)
        caches.append(cache)
    return np.stack(hs), np.stack(cs), caches


def layer_backward(dhs, dcT, caches, params, lap, K, H, gates="reference"):
    """Backprop through time of layer_forward.  dhs [T, N, M, H] = gradient of
    the outputs h_t, dcT = gradient of the final cell state (None = 0).
    Returns (dxs, dc0, dh0, dWx, dWh, db)."""
    Wx, Wh, _ = params
    T = len(caches)
    dh_rec = np.zeros_like(dhs[0], dtype=np.float64)
    dc = np.zeros_like(dh_rec) if dcT is None else np.asarray(dcT, np.float64)
    dWx = np.zeros(Wx.shape)
    dWh = np.zeros(Wh.shape)
    db = np.zeros(4 * H)
    dxs = [None] * T
    for t in range(T - 1, -1, -1):
        dx, dc, dh_rec, gWx, gWh, gb, _ = cell_backward(dhs[t] + dh_rec, dc, caches[t], Wx, Wh,
                                                        lap, K, H, gates)
        dxs[t] = dx
        dWx += gWx
        dWh += gWh
        db += gb
    return np.stack(dxs), dc, dh_rec, dWx, dWh, db


def unstack_time(x, T):
    """inference_glstm's input split (lib/gconv_lstm.py:272-275):
    [N, M, F*T] -> reshape [N, M, F, T] -> unstack axis 3 -> [T, N, M, F]."""
    N, M, C = x.shape
    return np.ascontiguousarray(np.moveaxis(x.reshape(N, M, C // T, T), 3, 0))
