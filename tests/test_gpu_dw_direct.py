"""k_dw_direct (dW = basis^T dy on registers only, no LDS batches) against
k_dw_slabs (CG_OPT_DW_DIRECT = 0): the per-chunk slabs -- and so dW -- bitwise equal
(same chunks, same row pairs in the same order per output element, same MFMA),
on the rows and planes layouts, every dy-width instantiation, ragged row
counts and column tails; and dW within 1e-5 of float64.  Reference: the
matmul gradient of lib/graph_conv.py:175."""
import numpy as np
import pytest

from oracle import cheb_oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev(built_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cnn_graph_amd import _lib
    _lib.lib()
    return torch.device("cuda", 0)


@pytest.mark.parametrize("R,FK,Fo", [(300001, 160, 32), (200003, 192, 64), (131072, 96, 128),
                                     (140001, 40, 256), (102400, 640, 32), (150000, 33, 30),
                                     (99999, 640, 2)])
def test_dw_direct_rows_bitwise(dev, cg_opts, R, FK, Fo):
    from cnn_graph_amd import ops
    g = torch.Generator(device=dev)
    g.manual_seed(R + FK + Fo)
    A = torch.randn((R, FK), device=dev, generator=g)
    D = torch.randn((R, Fo), device=dev, generator=g)
    cg_opts("dw_direct", "0")
    old = ops.weight_grad(A, D)
    cg_opts("dw_direct", "3")  # forced, whatever the wave count
    new = ops.weight_grad(A, D)
    torch.cuda.synchronize()
    assert torch.equal(new, old)
    ref = A.double().T @ D.double()
    assert O.normwise_err(new.cpu().numpy(), ref.cpu().numpy()) < 1e-5


@pytest.mark.parametrize("mode", ["3", "2"])
@pytest.mark.parametrize("R,Fin,K,Fo", [(200001, 64, 3, 64), (102400, 32, 20, 32), (80000, 16, 5, 128)])
def test_dw_direct_planes_bitwise(dev, cg_opts, mode, R, Fin, K, Fo):
    from cnn_graph_amd import ops
    g = torch.Generator(device=dev)
    g.manual_seed(R + K)
    st = R * Fin + 96
    buf = torch.randn((K * st,), device=dev, generator=g)
    D = torch.randn((R, Fo), device=dev, generator=g)
    planes = buf[:R * Fin].view(R, Fin)
    cg_opts("dw_direct", "0")
    old = ops.weight_grad_planes(planes, st, K, R, D)
    cg_opts("dw_direct", mode)
    new = ops.weight_grad_planes(planes, st, K, R, D)
    torch.cuda.synchronize()
    assert torch.equal(new, old)
    pl = torch.stack([buf[k * st:k * st + R * Fin].view(R, Fin) for k in range(K)]).double()
    ref = torch.einsum("krc,rg->ckg", pl, D.double()).reshape(Fin * K, Fo)
    assert O.normwise_err(new.cpu().numpy(), ref.cpu().numpy()) < 1e-5


@pytest.mark.parametrize("R,Fin,K", [(12 * 8 * 1024, 2, 3), (50001, 1, 1), (40000, 8, 4)])
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
    cg_opts("dw_direct", "0")
    old = ops.lstm_weight_grads(hpl, hst, xpl, xst, K, R, dpre)
    cg_opts("dw_direct", "3")  # forced, whatever the wave count
    new = ops.lstm_weight_grads(hpl, hst, xpl, xst, K, R, dpre)
    torch.cuda.synchronize()
    for a, b in zip(new, old):
        assert torch.equal(a, b)
    assert O.normwise_err(new[2].cpu().numpy(), dpre.double().sum(0).cpu().numpy()) < 1e-5


@pytest.mark.parametrize("R,FK,Fo", [(300001, 160, 32), (200003, 192, 64), (131072, 96, 128),
                                     (140001, 40, 256)])
def test_dw_direct_two_waves_bitwise(dev, cg_opts, R, FK, Fo):
    """The two-waves-per-SIMD build (CG_OPT_DW_W2 = 1, <= 256 registers) against the
    one-wave build and k_dw_slabs: dW bitwise equal (same chunks, same pairs,
    same MFMA sequence per output)."""
    from cnn_graph_amd import ops
    g = torch.Generator(device=dev)
    g.manual_seed(R + 7 * FK + Fo)
    A = torch.randn((R, FK), device=dev, generator=g)
    D = torch.randn((R, Fo), device=dev, generator=g)
    cg_opts("dw_direct", "0")
    ref = ops.weight_grad(A, D)
    out = {}
    for w2 in ("0", "1"):
        cg_opts("dw_direct", "3")
        cg_opts("dw_w2", w2)
        out[w2] = ops.weight_grad(A, D)
    torch.cuda.synchronize()
    assert torch.equal(out["0"], ref)
    assert torch.equal(out["1"], ref)


def test_dw_direct_two_waves_lstm_bitwise(dev, cg_opts):
    """cg_lstm_weight_grads (config E's shape class: H 32, Fin 2, K 3) on the
    two-waves build: dWh, dWx, db bitwise the one-wave build's."""
    from cnn_graph_amd import ops
    R, H, Fin, K = 12 * 8 * 1024, 32, 2, 3
    g = torch.Generator(device=dev)
    g.manual_seed(99)
    hst, xst = R * H + 96, R * Fin + 40
    hbuf = torch.randn((K * hst,), device=dev, generator=g)
    xbuf = torch.randn((K * xst,), device=dev, generator=g)
    dpre = torch.randn((R, 4 * H), device=dev, generator=g)
    hpl, xpl = hbuf[:R * H].view(R, H), xbuf[:R * Fin].view(R, Fin)
    out = {}
    for w2 in ("0", "1"):
        cg_opts("dw_direct", "3")
        cg_opts("dw_w2", w2)
        out[w2] = ops.lstm_weight_grads(hpl, hst, xpl, xst, K, R, dpre)
    torch.cuda.synchronize()
    for a, b in zip(out["0"], out["1"]):
        assert torch.equal(a, b)
