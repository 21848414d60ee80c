"""The ResGNN oracle (oracle/model_oracle.py) checked on the CPU: its
backward (TF-autodiff restatement) against central finite differences of its
own float64 loss (TF is absent -- TF boundary unpinned)."""
import numpy as np

from conftest import case, load_golden
from oracle import model_oracle as MO


def test_resgnn_oracle_gradients_match_finite_differences():
    c = case(load_golden("golden_A.npz"))
    lap = (c["Lt_rowptr"], c["Lt_col"], c["Lt_val"].astype(np.float64))
    rng = np.random.default_rng(0)
    N, M, Fin, F, K, R = 2, c["M"], 1, 3, 3, 1
    x = rng.standard_normal((N, M, Fin))
    labels = rng.standard_normal((N, M, 2))
    Ws = [rng.standard_normal((Fin * K, F)) * 0.5]
    for _ in range(R):
        Ws += [rng.standard_normal((F * K, F)) * 0.5, rng.standard_normal((F * K, F)) * 0.5]
    Ws.append(rng.standard_normal((F * K, 2)) * 0.5)
    out, cache = MO.forward(x, Ws, lap, K, R)
    _, dout = MO.loss_and_grad(out, labels)
    dWs = MO.backward(dout, cache, Ws, lap, K, R)

    def loss_of(Ws2):
        return MO.loss_and_grad(MO.forward(x, Ws2, lap, K, R)[0], labels)[0]

    eps = 1e-6
    for li, W in enumerate(Ws):
        for _ in range(5):
            idx = tuple(int(rng.integers(0, n)) for n in W.shape)
            Wp = [w.copy() for w in Ws]
            Wm = [w.copy() for w in Ws]
            Wp[li][idx] += eps
            Wm[li][idx] -= eps
            num = (loss_of(Wp) - loss_of(Wm)) / (2 * eps)
            assert abs(num - dWs[li][idx]) <= 1e-6 * max(1.0, abs(num)), (li, idx, num, dWs[li][idx])


def test_stacked_resgnn_oracle_gradients_match_finite_differences():
    """stack_num > 1 (lib/graph_conv.py:272-303): two channel groups, merge
    weights [M, 2] -- the backward against central differences of the loss."""
    c = case(load_golden("golden_A.npz"))
    lap = (c["Lt_rowptr"], c["Lt_col"], c["Lt_val"].astype(np.float64))
    rng = np.random.default_rng(1)
    N, M, C, F, K, R = 2, c["M"], 5, 3, 3, 1
    groups = [(0, 3), (3, 5)]
    x = rng.standard_normal((N, M, C))
    labels = rng.standard_normal((N, M, 2))

    def net(fin):
        Ws = [rng.standard_normal((fin * K, F)) * 0.5]
        for _ in range(R):
            Ws += [rng.standard_normal((F * K, F)) * 0.5, rng.standard_normal((F * K, F)) * 0.5]
        return Ws + [rng.standard_normal((F * K, 2)) * 0.5]

    nets = [net(b - a) for a, b in groups]
    merge = [rng.standard_normal((M, 2)) for _ in groups]
    X, caches = MO.stacked_forward(x, nets, merge, groups, lap, K, R)
    _, dX = MO.loss_and_grad(X, labels)
    dnets, dws = MO.stacked_backward(dX, caches, nets, merge, lap, K, R)

    def loss_of(nets2, merge2):
        return MO.loss_and_grad(MO.stacked_forward(x, nets2, merge2, groups, lap, K, R)[0], labels)[0]

    eps = 1e-6
    for i in range(len(groups)):
        for li in (0, len(nets[i]) - 1):
            idx = tuple(int(rng.integers(0, n)) for n in nets[i][li].shape)
            p = [[w.copy() for w in ws] for ws in nets]
            m = [[w.copy() for w in ws] for ws in nets]
            p[i][li][idx] += eps
            m[i][li][idx] -= eps
            num = (loss_of(p, merge) - loss_of(m, merge)) / (2 * eps)
            assert abs(num - dnets[i][li][idx]) <= 1e-6 * max(1.0, abs(num)), (i, li, idx)
        for _ in range(3):
            idx = (int(rng.integers(0, M)), int(rng.integers(0, 2)))
            p = [w.copy() for w in merge]
            m = [w.copy() for w in merge]
            p[i][idx] += eps
            m[i][idx] -= eps
            num = (loss_of(nets, p) - loss_of(nets, m)) / (2 * eps)
            assert abs(num - dws[i][idx]) <= 1e-6 * max(1.0, abs(num)), (i, idx)


def test_loss_ema_zero_debiased():
    """ExponentialMovingAverage(0.9) of a Tensor, zero-debiased: after one
    step the average equals the value; for a constant stream it stays there."""
    st = (0.0, 0.0, 0)
    st = MO.ema_update(st, 3.0)
    assert abs(st[1] - 3.0) < 1e-12
    st = MO.ema_update(st, 3.0)
    assert abs(st[1] - 3.0) < 1e-12
    st = MO.ema_update(st, 1.0)
    # biased after 3 steps: 0.1*(0.81*3 + 0.9*3 + 1) ; average = biased / (1 - 0.9**3)
    b = 0.1 * (0.81 * 3 + 0.9 * 3 + 1.0)
    assert abs(st[1] - b / (1 - 0.9 ** 3)) < 1e-12
