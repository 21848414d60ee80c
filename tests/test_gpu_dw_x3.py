"""k_dw_x3s (CG_OPT_DW_X3 = 1, the default for dW GEMMs with 65-128 dy
columns: dW = basis^T dy on the bf16 matrix pipe, every f32 operand split
exactly into three bf16 terms, dy staged once per chunk in LDS) against
float64 and against the f32-MFMA kernels (CG_OPT_DW_X3 = 0) on the same
inputs: within 1e-5 of float64, and no further from it than a small multiple
of the f32 kernel's own error -- on the rows and planes layouts, the
gconv-LSTM's one-pass weight gradients (x planes and the ones column, config
E's shape), ragged row counts and column tails.  Reference: the matmul
gradient of lib/graph_conv.py:175."""
import pytest

from oracle import cheb_oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

R_BIG = 1024 * 512  # >= 256 chunks of >= 256 rows: the x3 kernel's grid


@pytest.fixture(scope="module")
def dev(built_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cnn_graph_amd import _lib
    _lib.lib()
    return torch.device("cuda", 0)


def errs(new, old, ref):
    n = O.normwise_err(new.cpu().numpy(), ref.cpu().numpy())
    o = O.normwise_err(old.cpu().numpy(), ref.cpu().numpy())
    return n, o


def check(new, old, ref):
    n, o = errs(new, old, ref)
    assert n < 1e-5, (n, o)
    assert n <= 4 * o + 2e-7, (n, o)  # f32-accurate: no worse than the f32 MFMA chain
    assert not torch.equal(new, old)  # the bf16 kernel ran (other summation order)


def test_default_is_x3(dev):
    from cnn_graph_amd import _lib
    assert _lib.get_option("dw_x3") == 1


@pytest.mark.parametrize("R,FK,Fo", [(R_BIG + 1, 160, 128), (R_BIG + 3, 96, 96), (R_BIG + 7, 33, 124),
                                     (R_BIG + 4001, 250, 128), (R_BIG + 10, 40, 100), (R_BIG + 99, 64, 68)])
def test_dw_x3_rows(dev, cg_opts, R, FK, Fo):
    from cnn_graph_amd import ops
    g = torch.Generator(device=dev)
    g.manual_seed(R + FK + Fo)
    A = torch.randn((R, FK), device=dev, generator=g)
    D = torch.randn((R, Fo), device=dev, generator=g)
    cg_opts("dw_x3", 0)
    old = ops.weight_grad(A, D)
    cg_opts("dw_x3", 1)
    new = ops.weight_grad(A, D)
    torch.cuda.synchronize()
    check(new, old, A.double().T @ D.double())


@pytest.mark.parametrize("R,Fin,K,Fo", [(R_BIG + 1, 32, 3, 128), (R_BIG + 5, 16, 5, 96), (R_BIG + 2, 64, 3, 100)])
def test_dw_x3_planes(dev, cg_opts, R, Fin, K, Fo):
    from cnn_graph_amd import ops
    g = torch.Generator(device=dev)
    g.manual_seed(R + K)
    st = R * Fin + 96
    buf = torch.rand((K * st,), device=dev, generator=g)
    D = torch.randn((R, Fo), device=dev, generator=g)
    planes = buf[:R * Fin].view(R, Fin)
    cg_opts("dw_x3", 0)
    old = ops.weight_grad_planes(planes, st, K, R, D)
    cg_opts("dw_x3", 1)
    new = ops.weight_grad_planes(planes, st, K, R, D)
    torch.cuda.synchronize()
    pl = torch.stack([buf[k * st:k * st + R * Fin].view(R, Fin) for k in range(K)]).double()
    ref = torch.einsum("krc,rg->ckg", pl, D.double()).reshape(Fin * K, Fo)
    check(new, old, ref)


@pytest.mark.parametrize("R,Fin,K", [(12 * 128 * 1024, 2, 3), (R_BIG + 3, 1, 3), (R_BIG + 17, 8, 4)])
def test_dw_x3_lstm_weight_grads(dev, cg_opts, R, Fin, K):
    """cg_lstm_weight_grads' one pass (h planes, x planes, ones column; the
    first case is config E's T*N*M rows): dWh, dWx and db against float64 and
    the f32 kernel."""
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
    old = ops.lstm_weight_grads(hpl, hst, xpl, xst, K, R, dpre)
    cg_opts("dw_x3", 1)
    new = ops.lstm_weight_grads(hpl, hst, xpl, xst, K, R, dpre)
    torch.cuda.synchronize()
    d = dpre.double()
    hp = torch.stack([hbuf[k * hst:k * hst + R * H].view(R, H) for k in range(K)]).double()
    xp = torch.stack([xbuf[k * xst:k * xst + R * Fin].view(R, Fin) for k in range(K)]).double()
    refs = (torch.einsum("krc,rg->ckg", hp, d).reshape(H * K, 4 * H),
            torch.einsum("krc,rg->ckg", xp, d).reshape(Fin * K, 4 * H), d.sum(0))
    for a, b, r in zip(new, old, refs):
        n, o = errs(a, b, r)
        assert n < 1e-5 and n <= 4 * o + 2e-7, (n, o)


def test_dw_x3_exact_on_bf16_representable(dev):
    """Operands with <= 8 significant bits and small integer sums: the split
    has no mid / lo terms and every partial sum is exact, so dW equals the
    float64 product exactly (the lane maps and the store layout are right)."""
    from cnn_graph_amd import ops
    R, FK, Fo = R_BIG + 5, 160, 128
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    A = torch.randint(-8, 9, (R, FK), device=dev, generator=g).float()
    D = torch.randint(-8, 9, (R, Fo), device=dev, generator=g).float()
    new = ops.weight_grad(A, D)
    torch.cuda.synchronize()
    assert torch.equal(new.double(), A.double().T @ D.double())


def test_dw_x3_split_is_exact(dev):
    """Full-significand operands against one-hot dy rows: each output is ONE
    product a * 1 plus zeros, so the three terms must add back to a exactly --
    dW reproduces those basis entries bitwise."""
    from cnn_graph_amd import ops
    R, FK, Fo = R_BIG, 64, 128
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    A = torch.randn((R, FK), device=dev, generator=g) * 1e3
    D = torch.zeros((R, Fo), device=dev)
    rows = torch.arange(Fo, device=dev) * 4099  # one row per output column
    D[rows, torch.arange(Fo, device=dev)] = 1.0
    new = ops.weight_grad(A, D)
    torch.cuda.synchronize()
    assert torch.equal(new, A[rows].T)
