"""The gconv-LSTM oracle (oracle/lstm_oracle.py) checked on the CPU.

TensorFlow is absent, so the cell's TF-autodiff gradient has no golden
vectors ("TF boundary unpinned").  The oracle's backprop
through time is therefore pinned to its own forward by central finite
differences in float64, and its convolutions are the pinned cheb_oracle ones
(whose fp32 basis is bit-equal to lib/graph.py::chebyshev on the golden
fixtures)."""
import numpy as np
import pytest

from conftest import case, load_golden
from oracle import cheb_oracle as O
from oracle import lstm_oracle as L


def _setup(gates, seed=0, T=3, N=2, Fin=2, H=3, K=3):
    c = case(load_golden("golden_A.npz"))
    lap = (c["Lt_rowptr"], c["Lt_col"], c["Lt_val"].astype(np.float64))
    M = c["M"]
    rng = np.random.default_rng(seed)
    xs = rng.standard_normal((T, N, M, Fin))
    Wx = rng.uniform(-0.3, 0.3, (K * Fin, 4 * H))
    Wh = rng.uniform(-0.3, 0.3, (K * H, 4 * H))
    b = rng.uniform(-0.5, 0.5, 4 * H)
    c0 = rng.standard_normal((N, M, H)) * 0.5
    h0 = rng.standard_normal((N, M, H)) * 0.5
    gh = rng.standard_normal((T, N, M, H))     # dLoss/dh_t
    gc = rng.standard_normal((N, M, H))        # dLoss/dc_T
    return dict(lap=lap, xs=xs, params=[Wx, Wh, b], c0=c0, h0=h0, gh=gh, gc=gc, K=K, H=H,
                gates=gates)


def _loss(s, xs=None, params=None, c0=None, h0=None):
    xs = s["xs"] if xs is None else xs
    params = s["params"] if params is None else params
    c0 = s["c0"] if c0 is None else c0
    h0 = s["h0"] if h0 is None else h0
    hs, cs, _ = L.layer_forward(xs, params, s["lap"], s["K"], s["H"], c0, h0, s["gates"])
    return float((hs * s["gh"]).sum() + (cs[-1] * s["gc"]).sum())


def _fd(f, a, idx, eps=1e-6):
    a = a.copy()
    a0 = a[idx]
    a[idx] = a0 + eps
    fp = f(a)
    a[idx] = a0 - eps
    fm = f(a)
    return (fp - fm) / (2 * eps)


@pytest.mark.parametrize("gates", ["reference", "standard"])
def test_bptt_matches_finite_differences(gates):
    s = _setup(gates)
    hs, cs, caches = L.layer_forward(s["xs"], s["params"], s["lap"], s["K"], s["H"], s["c0"],
                                     s["h0"], gates)
    dxs, dc0, dh0, dWx, dWh, db = L.layer_backward(s["gh"], s["gc"], caches, s["params"], s["lap"],
                                                   s["K"], s["H"], gates)
    rng = np.random.default_rng(1)
    Wx, Wh, b = s["params"]
    checks = [
        ("Wx", dWx, Wx, lambda a: _loss(s, params=[a, Wh, b])),
        ("Wh", dWh, Wh, lambda a: _loss(s, params=[Wx, a, b])),
        ("b", db, b, lambda a: _loss(s, params=[Wx, Wh, a])),
        ("xs", dxs, s["xs"], lambda a: _loss(s, xs=a)),
        ("c0", dc0, s["c0"], lambda a: _loss(s, c0=a)),
        ("h0", dh0, s["h0"], lambda a: _loss(s, h0=a)),
    ]
    for name, g, a, f in checks:
        for _ in range(6):
            idx = tuple(int(rng.integers(0, n)) for n in a.shape)
            num = _fd(f, a, idx)
            assert abs(num - g[idx]) <= 1e-6 * max(1.0, abs(num)), (name, idx, num, g[idx])


def test_cell_gate_functions_follow_the_reference():
    """z = tan and o = tanh under gates='reference' (lib/gconv_lstm.py:188, :209)."""
    s = _setup("reference", T=1, N=1)
    Wx, Wh, b = s["params"]
    H = s["H"]
    x, c, h = s["xs"][0], s["c0"], s["h0"]
    cn, hn, cache = L.cell_forward(x, c, h, Wx, Wh, b, s["lap"], s["K"], H, "reference")
    _, gx = L.cheb_conv64(x, s["lap"], Wx, s["K"])
    _, gh = L.cheb_conv64(h, s["lap"], Wh, s["K"])
    a = gx + gh + b
    sig = lambda v: 1 / (1 + np.exp(-v))  # noqa: E731
    z, i, f, o = np.tan(a[..., :H]), sig(a[..., H:2 * H]), sig(a[..., 2 * H:3 * H]), np.tanh(a[..., 3 * H:])
    np.testing.assert_allclose(cn, f * c + i * z, rtol=1e-14)
    np.testing.assert_allclose(hn, o * np.tanh(f * c + i * z), rtol=1e-14)


def test_cheb_conv64_is_the_pinned_basis_in_float64():
    """Rounded to fp32 inputs, cheb_conv64's basis agrees with the fp32
    reference-order basis to fp32 precision."""
    c = case(load_golden("golden_A.npz"))
    lap = (c["Lt_rowptr"], c["Lt_col"], c["Lt_val"])
    A64, y64 = L.cheb_conv64(c["x"].astype(np.float64), lap, c["W"], c["K"])
    assert O.normwise_err(A64, c["basis"]) < 1e-6
    assert O.normwise_err(y64, c["y_ref"]) < 1e-6


def test_unstack_time_matches_reshape_unstack():
    x = np.arange(2 * 3 * 8, dtype=np.float64).reshape(2, 3, 8)  # F=2, T=4
    xs = L.unstack_time(x, 4)
    assert xs.shape == (4, 2, 3, 2)
    for t in range(4):
        np.testing.assert_array_equal(xs[t], x.reshape(2, 3, 2, 4)[..., t])
