"""The Fourier filter (lib/graph_conv.py:83-111), bias/activation (:178-199),
fc (:220-226) and the pooled multi-level cgcnn (lib/models.py:61-127) on the
GPU through the C ABI vs the float64 oracles.  Bar: 1e-5 max-abs-normalised."""
import numpy as np
import pytest
import scipy.sparse

from conftest import case, load_golden
from oracle import cheb_oracle as O
from oracle import fourier_oracle as FO
from oracle.lstm_oracle import cheb_conv64

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


def t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(dev)


def f64(x):
    return x.detach().cpu().numpy().astype(np.float64)


def r32(a):
    return np.asarray(a, np.float32).astype(np.float64)


def golden_L(name):
    c = case(load_golden(name))
    M = c["M"]
    Lt = scipy.sparse.csr_matrix((c["Lt_val"], c["Lt_col"], c["Lt_rowptr"]), shape=(M, M))
    return (Lt + scipy.sparse.identity(M, dtype=np.float32, format="csr")).tocsr()


@pytest.mark.parametrize("name,N,Fin,Fout", [("golden_A.npz", 4, 1, 1), ("golden_A.npz", 3, 3, 5),
                                             ("golden_E.npz", 2, 2, 32), ("golden_B.npz", 8, 1, 32)])
def test_fourier_forward_backward_vs_oracle(dev, name, N, Fin, Fout):
    from cnn_graph_amd import graph, ops
    L = golden_L(name)
    M = L.shape[0]
    _, U = graph.fourier(L)                      # lib/graph.py:148 on the fp32 Laplacian
    rng = np.random.default_rng(N * 100 + Fin * 10 + Fout)
    x = rng.standard_normal((N, M, Fin)).astype(np.float32)
    W = (rng.standard_normal((M, Fout, Fin)) * 0.1).astype(np.float32)
    dy = rng.standard_normal((N, M, Fout)).astype(np.float32)
    xt = t(x, dev).requires_grad_(True)
    Wt = t(W, dev).requires_grad_(True)
    y = ops.fourier_conv(xt, Wt, t(U, dev))
    y.backward(t(dy, dev))
    torch.cuda.synchronize()
    ry, xhat = FO.fourier_forward(r32(x), r32(W), r32(U))
    rdx, rdW = FO.fourier_backward(r32(dy), r32(W), r32(U), xhat)
    assert O.normwise_err(f64(y), ry) < TOL
    assert O.normwise_err(f64(xt.grad), rdx) < TOL
    assert O.normwise_err(f64(Wt.grad), rdW) < TOL


def test_graphconv_fourier_filter_by_name(dev):
    """GraphConv(filter='fourier') binds the spectral filter by name
    (lib/graph_conv.py:74) with W [M, Fout, Fin] in its variable scope;
    filter.fourier_conv (lib/filter.py:30-42) gives the same output."""
    from cnn_graph_amd import filter as cfilter
    from cnn_graph_amd import graph
    from cnn_graph_amd.graph_conv import GraphConv
    L = golden_L("golden_A.npz")
    M = L.shape[0]
    gc = GraphConv(filter="fourier", device=dev)
    rng = np.random.default_rng(5)
    x = rng.standard_normal((2, M, 2)).astype(np.float32)
    with gc.variable_scope("conv1"):
        y = gc.filter(t(x, dev), L, 3, 5)
    W = gc.weights["conv1/weights"]
    assert tuple(W.shape) == (M, 3, 2)
    assert float(W.abs().max()) <= 0.2
    _, U = graph.fourier(L)
    ry, _ = FO.fourier_forward(r32(x), f64(W), r32(U))
    assert O.normwise_err(f64(y), ry) < TOL
    y2 = cfilter.fourier_conv(t(x, dev), L, 2, 3, 5, W=W)
    assert O.normwise_err(f64(y2), ry) < TOL


@pytest.mark.parametrize("act", ["relu", "tanh", "none"])
@pytest.mark.parametrize("bshape", [None, (1, 1, 16), (1, 100, 16)])
def test_bias_act_vs_oracle(dev, act, bshape):
    from cnn_graph_amd import ops
    rng = np.random.default_rng(7)
    x = rng.standard_normal((5, 100, 16)).astype(np.float32)
    dy = rng.standard_normal(x.shape).astype(np.float32)
    xt = t(x, dev).requires_grad_(True)
    b = bt = None
    if bshape is not None:
        b = rng.standard_normal(bshape).astype(np.float32)
        bt = t(b, dev).requires_grad_(True)
    y = ops.bias_act(xt, bt, act)
    y.backward(t(dy, dev))
    torch.cuda.synchronize()
    ry = FO.bias_act(r32(x), None if b is None else r32(b), act)
    rdz, rdb = FO.bias_act_backward(r32(dy), f64(y), act, bshape)
    assert O.normwise_err(f64(y), ry) < TOL
    assert O.normwise_err(f64(xt.grad), rdz) < TOL
    if bshape is not None:
        assert O.normwise_err(f64(bt.grad), rdb) < TOL


def test_graphconv_b1tanh_b2relu_fc(dev):
    """b1tanh / b2relu create their bias (constant 0.1) in the current scope;
    fc = relu(x W + b) on the MFMA GEMM; gradients through autograd."""
    from cnn_graph_amd.graph_conv import GraphConv
    gc = GraphConv(device=dev)
    rng = np.random.default_rng(11)
    x = rng.standard_normal((6, 40, 8)).astype(np.float32)
    with gc.variable_scope("a"):
        y1 = gc.b1tanh(t(x, dev))
    with gc.variable_scope("b"):
        y2 = gc.b2relu(t(x, dev))
    assert tuple(gc.weights["a/bias"].shape) == (1, 1, 8)
    assert tuple(gc.weights["b/bias"].shape) == (1, 40, 8)
    b01 = np.float64(np.float32(0.1))
    assert O.normwise_err(f64(y1), np.tanh(r32(x) + b01)) < TOL
    assert O.normwise_err(f64(y2), np.maximum(r32(x) + b01, 0)) < TOL
    xf = t(rng.standard_normal((37, 70)), dev).requires_grad_(True)
    with gc.variable_scope("fc1"):
        z = gc.fc(xf, 45)
    Wf, bf = gc.weights["fc1/weights"], gc.weights["fc1/bias"]
    dz = rng.standard_normal((37, 45)).astype(np.float32)
    z.backward(t(dz, dev))
    torch.cuda.synchronize()
    xn = f64(xf)
    pre = xn @ f64(Wf) + f64(bf)
    assert O.normwise_err(f64(z), np.maximum(pre, 0)) < TOL
    g = r32(dz) * (pre > 0)
    assert O.normwise_err(f64(Wf.grad), xn.T @ g) < TOL
    assert O.normwise_err(f64(bf.grad), g.sum(0)) < TOL
    assert O.normwise_err(f64(xf.grad), g @ f64(Wf).T) < TOL


@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False), (True, True)])
def test_gemm_transposes(dev, ta, tb):
    from cnn_graph_amd import ops
    rng = np.random.default_rng(int(ta) * 2 + int(tb))
    M, N, K = 67, 129, 300
    a = rng.standard_normal((K, M) if ta else (M, K)).astype(np.float32)
    b = rng.standard_normal((N, K) if tb else (K, N)).astype(np.float32)
    c = ops.gemm(t(a, dev), t(b, dev), trans_a=ta, trans_b=tb)
    torch.cuda.synchronize()
    ref = (r32(a).T if ta else r32(a)) @ (r32(b).T if tb else r32(b))
    assert O.normwise_err(f64(c), ref) < TOL


def test_cgcnn_pooled_mnist_pyramid_vs_oracle(dev):
    """usage.ipynb's architecture (F=[32, 64], K=[20, 20], p=[4, 2], M=[512, 10])
    on the reference's own MNIST coarsening pyramid (golden_B visit orders):
    conv1 on L0 (976), mpool 4, conv2 on L2 (244), mpool 2, fc1, logits."""
    from cnn_graph_amd import coarsening, graph
    from cnn_graph_amd.graph_conv import GraphConv
    from cnn_graph_amd.plan import plan_for
    g = load_golden("golden_B.npz")
    A = scipy.sparse.csr_matrix((g["A_data"], g["A_indices"], g["A_indptr"]), shape=tuple(g["A_shape"]))
    graphs, perm = coarsening.coarsen(A, 4, rids=[g[f"rid{i}"] for i in range(4)], verbose=False)
    L = [graph.laplacian(G, normalized=True) for G in graphs]
    F, K, p, Mfc = [32, 64], [20, 20], [4, 2], [512, 10]
    N = 8
    rng = np.random.default_rng(3)
    x = coarsening.perm_data(rng.random((N, A.shape[0])), perm).astype(np.float32)
    gc = GraphConv(filter="chebyshev5", brelu="b1relu", pool="mpool1", device=dev)
    out = gc.cgcnn_inference(t(x, dev), L, F, K, p, Mfc)
    torch.cuda.synchronize()
    assert tuple(out.shape) == (N, 10)
    Ls = GraphConv.select_laplacians(L, p)
    h = r32(x)[:, :, None]
    for i in range(2):
        pl = plan_for(Ls[i], lmax=2, device=0)
        lap = (pl.rowptr, pl.col, pl.val.astype(np.float64))
        _, y = cheb_conv64(h, lap, f64(gc.weights[f"conv{i + 1}/weights"]), K[i])
        h, _ = O.mpool1_forward(np.maximum(y, 0), p[i])
    h = h.reshape(N, -1)
    h = np.maximum(h @ f64(gc.weights["fc1/weights"]) + f64(gc.weights["fc1/bias"]), 0)
    ref = h @ f64(gc.weights["logits/weights"]) + f64(gc.weights["logits/bias"])
    assert O.normwise_err(f64(out), ref) < TOL
