"""CPU oracle for the spectral (Fourier) filter and the dense layers around the
graph filters.

TEST INFRASTRUCTURE ONLY (same contract as ``cheb_oracle``): imported by
``tests/`` as the checker, never by ``cnn_graph_amd/``.

Float64 restatement, from the reference source text (TensorFlow is not
installed here, so the TF boundary is unpinned and truth is float64 NumPy):
  * ``filter_in_fourier`` lib/graph_conv.py:83-99 and ``fourier`` :101-111
    (dupes lib/models.py:129-159) with U = eigenvectors of L from
    ``graph.fourier`` (lib/graph.py:148-166);
  * ``b1tanh`` / ``b2relu`` :189-199 and ``fc`` :220-226.
"""
from __future__ import annotations

import numpy as np


def fourier_forward(x, W, U):
    """filter_in_fourier, lib/graph_conv.py:83-99.

    x [N, M, Fin]; W [M, Fout, Fin]; U [M, M] with eigenvectors in columns
    (the reference passes ``U.T`` as its constant ``U``, :108, so its
    ``matmul(U, x)`` at :90 is U^T x and ``matmul(x, U)`` at :97 is x U^T).
    Returns (y [N, M, Fout], xhat [N, Fin, M])."""
    x = np.asarray(x, np.float64)
    W = np.asarray(W, np.float64)
    U = np.asarray(U, np.float64)
    N, M, Fin = x.shape
    x0 = np.transpose(x, (1, 2, 0)).reshape(M, Fin * N)          # :87-89
    xh = (U.T @ x0).reshape(M, Fin, N)                           # :90-91
    yh = np.matmul(W, xh)                                        # :93  M x Fout x N
    Fout = W.shape[1]
    yh = np.transpose(yh).reshape(N * Fout, M)                   # :94-95 N x Fout x M
    y = (yh @ U.T).reshape(N, Fout, M)                           # :97-98
    xhat = np.transpose(xh, (2, 1, 0))                           # N x Fin x M
    return np.ascontiguousarray(np.transpose(y, (0, 2, 1))), np.ascontiguousarray(xhat)


def fourier_backward(dy, W, U, xhat):
    """TF autodiff of fourier_forward: (dx [N, M, Fin], dW [M, Fout, Fin])."""
    dy = np.asarray(dy, np.float64)
    W = np.asarray(W, np.float64)
    U = np.asarray(U, np.float64)
    xhat = np.asarray(xhat, np.float64)
    # dYh[n, o, m] = sum_v dy[n, v, o] U[v, m]
    dYh = np.einsum("nvo,vm->nom", dy, U)
    dW = np.einsum("nom,nim->moi", dYh, xhat)
    dXh = np.einsum("moi,nom->nim", W, dYh)
    dx = np.einsum("nim,vm->nvi", dXh, U)
    return dx, dW


def bias_act(x, b, act):
    """x + b (broadcast) then relu / tanh / identity: b1tanh, b2relu, fc."""
    z = np.asarray(x, np.float64) + (0.0 if b is None else np.asarray(b, np.float64))
    if act == "relu":
        return np.maximum(z, 0.0)
    if act == "tanh":
        return np.tanh(z)
    return z


def bias_act_backward(dy, y, act, bshape):
    """(dz, db) for y = act(x + b); db summed over the broadcast axes."""
    dy = np.asarray(dy, np.float64)
    y = np.asarray(y, np.float64)
    if act == "relu":
        dz = dy * (y > 0)
    elif act == "tanh":
        dz = dy * (1.0 - y * y)
    else:
        dz = dy
    db = None
    if bshape is not None:
        axes = tuple(i for i in range(dz.ndim) if i < dz.ndim - len(bshape) or
                     bshape[i - (dz.ndim - len(bshape))] == 1)
        db = dz.sum(axis=axes).reshape(bshape)
    return dz, db
