"""Filters wider than 256 output channels (k_dw_slabs stages at most
256 dy columns per row, so wider outputs run as 256-column slices).  The
reference sets no upper bound on Fout (lib/graph_conv.py:174 `[Fin*K, Fout]`,
the gconv-LSTM's 4*num_hidden gate columns, lib/gconv_lstm.py:600-627).
dW / dx within 1e-5 of float64; the slices' slabs bitwise equal to the
unsliced kernel on the columns it covers."""
import numpy as np
import pytest
import scipy.sparse

from conftest import case, load_golden
from oracle import cheb_oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

TOL = 1e-5


@pytest.fixture(scope="module")
def dev(built_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cnn_graph_amd import _lib
    _lib.lib()
    return torch.device("cuda", 0)


@pytest.mark.parametrize("FK,Fo", [(96, 512), (40, 300), (33, 257)])
def test_weight_grad_wide_fout(dev, FK, Fo):
    from cnn_graph_amd import ops
    g = torch.Generator(device=dev)
    g.manual_seed(FK + Fo)
    R = 5000
    A = torch.randn((R, FK), device=dev, generator=g)
    D = torch.randn((R, Fo), device=dev, generator=g)
    got = ops.weight_grad(A, D)
    first = ops.weight_grad(A, D[:, :256].contiguous())  # one slice, unsliced kernel
    torch.cuda.synchronize()
    ref = A.double().cpu().T @ D.double().cpu()
    assert O.normwise_err(got.cpu().numpy(), ref.numpy()) < TOL
    assert torch.equal(got[:, :256], first)


def test_weight_grad_planes_wide_fout(dev):
    from cnn_graph_amd import ops
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    R, Fin, K, Fo = 4096, 16, 3, 512
    st = R * Fin + 64
    buf = torch.randn((K * st,), device=dev, generator=g)
    D = torch.randn((R, Fo), device=dev, generator=g)
    got = ops.weight_grad_planes(buf[:R * Fin].view(R, Fin), st, K, R, D)
    torch.cuda.synchronize()
    pl = torch.stack([buf[k * st:k * st + R * Fin].view(R, Fin) for k in range(K)]).double().cpu()
    ref = torch.einsum("krc,rg->ckg", pl, D.double().cpu()).reshape(Fin * K, Fo)
    assert O.normwise_err(got.cpu().numpy(), ref.numpy()) < TOL


def test_cheb_backward_fout_512_vs_oracle(dev):
    """chebyshev5 forward + backward with Fout = 512 on config E's graph."""
    from cnn_graph_amd import ops
    from cnn_graph_amd.plan import ChebPlan
    c = case(load_golden("golden_E.npz"))
    M = c["M"]
    plan = ChebPlan(scipy.sparse.csr_matrix((c["Lt_val"], c["Lt_col"], c["Lt_rowptr"]),
                                            shape=(M, M)), device=0)
    rng = np.random.default_rng(11)
    N, Fin, K, Fout = 4, 4, 3, 512
    x = rng.random((N, M, Fin), dtype=np.float32)
    W = (rng.standard_normal((Fin * K, Fout)) * 0.1).astype(np.float32)
    dy = rng.standard_normal((N, M, Fout)).astype(np.float32)
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    basis, y = ops.cheb_forward(plan, tt(x), tt(W), K)
    dx, dW = ops.cheb_backward(plan, tt(dy), basis, tt(W), K)
    torch.cuda.synchronize()
    rp, ci, v = c["Lt_rowptr"], c["Lt_col"], c["Lt_val"]
    ob, oy = O.cheb_forward(x, rp, ci, v, W, K)
    assert O.normwise_err(y.cpu().numpy(), oy) < TOL
    odx, odW = O.cheb_backward(dy, ob, W, rp, ci, v, N, M, Fin, K)
    assert O.normwise_err(dx.cpu().numpy(), odx) < TOL
    assert O.normwise_err(dW.cpu().numpy(), odW) < TOL
