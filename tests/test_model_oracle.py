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
