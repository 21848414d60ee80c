"""k_dw_direct (dW = basis^T dy on registers only, no LDS batches; the
default wherever its grid fills the chip: >= 1 024 waves, i.e. >= 1 024 chunks
of >= 512 rows) against k_dw_slabs (CG_OPT_DW_DIRECT = 0): the per-chunk slabs
-- and so dW -- bitwise equal (same chunks, same row pairs in the same order
per output element, same MFMA), on the rows and planes layouts, every
dy-width instantiation, ragged row counts and column tails; and dW within 1e-5
of float64.  Reference: the matmul gradient of lib/graph_conv.py:175.

Round 6: the forced modes (CG_OPT_DW_DIRECT 2 / 3) and the one-wave builds
(CG_OPT_DW_W2 = 0) live in the ablation build only, so these tests run the
default kernel at row counts where it is the one chosen."""
import numpy as np
import pytest

from oracle import cheb_oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

R_BIG = 1024 * 512  # rows from which every chunk is >= 512 rows and 1 024 chunks fill the chip


@pytest.fixture(scope="module")
def dev(built_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cnn_graph_amd import _lib
    _lib.lib()
    return torch.device("cuda", 0)


@pytest.mark.parametrize("R,FK,Fo", [(R_BIG + 1, 160, 32), (R_BIG + 3, 192, 64), (R_BIG, 96, 128),
                                     (R_BIG + 4001, 40, 256), (R_BIG + 7, 640, 32), (R_BIG + 10, 33, 30),
                                     (R_BIG + 99, 640, 2)])
def test_dw_direct_rows_bitwise(dev, cg_opts, R, FK, Fo):
    from cnn_graph_amd import ops
    g = torch.Generator(device=dev)
    g.manual_seed(R + FK + Fo)
    A = torch.randn((R, FK), device=dev, generator=g)
    D = torch.randn((R, Fo), device=dev, generator=g)
    cg_opts("dw_x3", 0)  # the f32 kernels (k_dw_x3s: tests/test_gpu_dw_x3.py)
    cg_opts("dw_direct", "0")
    old = ops.weight_grad(A, D)
    cg_opts("dw_direct", "1")  # the default: k_dw_direct at this size
    new = ops.weight_grad(A, D)
    torch.cuda.synchronize()
    assert torch.equal(new, old)
    ref = A.double().T @ D.double()
    assert O.normwise_err(new.cpu().numpy(), ref.cpu().numpy()) < 1e-5


@pytest.mark.parametrize("R,Fin,K,Fo", [(R_BIG + 1, 64, 3, 64), (R_BIG + 5, 32, 20, 32), (R_BIG + 2, 16, 5, 128)])
def test_dw_direct_planes_bitwise(dev, cg_opts, R, Fin, K, Fo):
    from cnn_graph_amd import ops
    g = torch.Generator(device=dev)
    g.manual_seed(R + K)
    st = R * Fin + 96
    buf = torch.randn((K * st,), device=dev, generator=g)
    D = torch.randn((R, Fo), device=dev, generator=g)
    planes = buf[:R * Fin].view(R, Fin)
    cg_opts("dw_x3", 0)
    cg_opts("dw_direct", "0")
    old = ops.weight_grad_planes(planes, st, K, R, D)
    cg_opts("dw_direct", "1")
    new = ops.weight_grad_planes(planes, st, K, R, D)
    torch.cuda.synchronize()
    assert torch.equal(new, old)
    pl = torch.stack([buf[k * st:k * st + R * Fin].view(R, Fin) for k in range(K)]).double()
    ref = torch.einsum("krc,rg->ckg", pl, D.double()).reshape(Fin * K, Fo)
    assert O.normwise_err(new.cpu().numpy(), ref.cpu().numpy()) < 1e-5


@pytest.mark.parametrize("R,Fin,K", [(12 * 48 * 1024, 2, 3), (R_BIG + 1, 1, 1), (R_BIG + 3, 8, 4)])
def test_dw_direct_lstm_weight_grads_bitwise(dev, cg_opts, R, Fin, K):
    """cg_lstm_weight_grads' one pass (h planes, x planes and the ones column
    of the bias) on the direct kernel: dWh, dWx, db bitwise k_dw_slabs'."""
    from cnn_graph_amd import ops
    H = 32
    g = torch.Generator(device=dev)
    g.manual_seed(R + Fin)
    hst, xst = R * H + 96, R * Fin + 40
    hbuf = torch.randn((K * hst,), device=dev, generator=g)
    xbuf = torch.randn((K * xst,), device=dev, generator=g)
    dpre = torch.randn((R, 4 * H), device=dev, generator=g)
    hpl, xpl = hbuf[:R * H].view(R, H), xbuf[:R * Fin].view(R, Fin)
    cg_opts("dw_x3", 0)
    cg_opts("dw_direct", "0")
    old = ops.lstm_weight_grads(hpl, hst, xpl, xst, K, R, dpre)
    cg_opts("dw_direct", "1")
    new = ops.lstm_weight_grads(hpl, hst, xpl, xst, K, R, dpre)
    torch.cuda.synchronize()
    for a, b in zip(new, old):
        assert torch.equal(a, b)
    assert O.normwise_err(new[2].cpu().numpy(), dpre.double().sum(0).cpu().numpy()) < 1e-5


def test_release_rejects_ablation_only_values(dev, cg_opts):
    """The forced direct modes and the one-wave builds are ablation-build
    options: the release library refuses them."""
    from cnn_graph_amd import _lib
    for name, v in (("dw_direct", 2), ("dw_direct", 3), ("dw_w2", 0)):
        with pytest.raises(_lib.CGError):
            cg_opts(name, v)
