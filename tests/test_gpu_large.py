"""Large graphs on the streaming path.

  C: the reference's own 10 000-vertex cosine 16-NN graph (golden_C.npz, made
     by importing lib/graph.py): basis bit-exact to lib/graph.py::chebyshev,
     y / dx / dW within 1e-5 of the float64 truth; full layer-1 batch (N=128)
     and a Fin=32 layer-2 shape against the oracle.
  D: the seeded Chung-Lu power-law graph (scripts/synth_graphs.py, M = 2^18,
     nnz(L~) = 4 189 524, rows up to 1 131 nnz) with Fin = Fout = 64, K = 3:
     one sample against the oracle (whose SpMM order is pinned to the
     reference's, tests/test_oracle_golden.py), and batch-size-independent
     identities at a larger batch (per-sample independence, linearity).
"""
import os
import sys

import numpy as np
import pytest
import scipy.sparse

from conftest import ROOT, case, load_golden
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


def t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def plan_of(rp, ci, v, M, path="auto"):
    from cnn_graph_amd.plan import ChebPlan
    return ChebPlan(scipy.sparse.csr_matrix((v, ci, rp), shape=(M, M)), device=0, path=path)


@pytest.fixture(scope="module")
def graph_c():
    return case(load_golden("golden_C.npz"))


@pytest.fixture(scope="module")
def graph_d():
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import synth_graphs
    from cnn_graph_amd.graph import canonical_csr, rescale_L
    rp, ci, v = canonical_csr(rescale_L(synth_graphs.config_d_laplacian(), 2))
    return rp, ci, v, len(rp) - 1


@pytest.mark.parametrize("prefix", ["", "fin3_"])
def test_config_c_golden(dev, graph_c, prefix):
    from cnn_graph_amd import ops
    g = load_golden("golden_C.npz")
    c = case(g, prefix)
    M = graph_c["M"]
    plan = plan_of(graph_c["Lt_rowptr"], graph_c["Lt_col"], graph_c["Lt_val"], M)
    assert plan.query_path(c["N"], c["Fin"], c["K"], c["Fout"]) == "stream"
    basis, y = ops.cheb_forward(plan, t(c["x"], dev), t(c["W"], dev), c["K"])
    dx, dW = ops.cheb_backward(plan, t(c["dy"], dev), basis, t(c["W"], dev), c["K"])
    torch.cuda.synchronize()
    assert np.array_equal(basis.cpu().numpy(), c["basis"]), "basis not bit-exact to lib/graph.py"
    assert O.normwise_err(y.cpu().numpy(), c["y_ref"]) < TOL
    assert O.normwise_err(dx.cpu().numpy(), c["dx_ref"]) < TOL
    assert O.normwise_err(dW.cpu().numpy(), c["dW_ref"]) < TOL


@pytest.mark.parametrize("N,Fin,K,Fout", [(128, 1, 5, 32), (8, 32, 5, 32)])
def test_config_c_batch_vs_oracle(dev, graph_c, N, Fin, K, Fout):
    """Config C layer 1 at its full batch (N=128) and a layer-2 shape (Fin=32)."""
    from cnn_graph_amd import ops
    rp, ci, v, M = graph_c["Lt_rowptr"], graph_c["Lt_col"], graph_c["Lt_val"], graph_c["M"]
    rng = np.random.default_rng(N + Fin)
    x = rng.random((N, M, Fin), dtype=np.float32)
    W = (rng.standard_normal((Fin * K, Fout)) * 0.1).astype(np.float32)
    dy = rng.standard_normal((N, M, Fout)).astype(np.float32)
    plan = plan_of(rp, ci, v, M)
    basis, y = ops.cheb_forward(plan, t(x, dev), t(W, dev), K)
    dx, dW = ops.cheb_backward(plan, t(dy, dev), basis, t(W, dev), K)
    torch.cuda.synchronize()
    ob, oy = O.cheb_forward(x, rp, ci, v, W, K)
    assert np.array_equal(basis.cpu().numpy(), ob)
    assert O.normwise_err(y.cpu().numpy(), oy) < TOL
    odx, odW = O.cheb_backward(dy, ob, W, rp, ci, v, N, M, Fin, K)
    assert O.normwise_err(dx.cpu().numpy(), odx) < TOL
    assert O.normwise_err(dW.cpu().numpy(), odW) < TOL


def test_config_d_one_sample_vs_oracle(dev, graph_d):
    """Config D shape (Fin = Fout = 64, K = 3) on the 2^18-vertex power-law graph."""
    from cnn_graph_amd import ops
    rp, ci, v, M = graph_d
    N, Fin, K, Fout = 1, 64, 3, 64
    rng = np.random.default_rng(11)
    x = rng.random((N, M, Fin), dtype=np.float32)
    W = (rng.standard_normal((Fin * K, Fout)) * 0.1).astype(np.float32)
    dy = rng.standard_normal((N, M, Fout)).astype(np.float32)
    plan = plan_of(rp, ci, v, M)
    assert plan.query_path(N, Fin, K, Fout) == "stream"
    basis, y = ops.cheb_forward(plan, t(x, dev), t(W, dev), K)
    dx, dW = ops.cheb_backward(plan, t(dy, dev), basis, t(W, dev), K)
    torch.cuda.synchronize()
    ob, oy = O.cheb_forward(x, rp, ci, v, W, K)
    assert np.array_equal(basis.cpu().numpy(), ob)
    assert O.normwise_err(y.cpu().numpy(), oy) < TOL
    odx, odW = O.cheb_backward(dy, ob, W, rp, ci, v, N, M, Fin, K)
    assert O.normwise_err(dx.cpu().numpy(), odx) < TOL
    assert O.normwise_err(dW.cpu().numpy(), odW) < TOL


def test_config_d_batch_identities(dev, graph_d):
    """At N=16 (B = 1 024 dense columns): each sample's basis is bitwise the
    one it gets alone (per-sample independence of the filter), and the filter
    is linear: y(2 x1 + x2) = 2 y(x1) + y(x2) to fp32 rounding."""
    from cnn_graph_amd import ops
    rp, ci, v, M = graph_d
    N, Fin, K, Fout = 16, 64, 3, 64
    plan = plan_of(rp, ci, v, M)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    x1 = torch.rand((N, M, Fin), device=dev, generator=g)
    x2 = torch.rand((N, M, Fin), device=dev, generator=g)
    W = torch.randn((Fin * K, Fout), device=dev, generator=g) * 0.1
    b1, y1 = ops.cheb_forward(plan, x1, W, K)
    bs, ys = ops.cheb_forward(plan, x1[5:6].contiguous(), W, K)
    torch.cuda.synchronize()
    assert torch.equal(b1.view(N, M, Fin * K)[5], bs.view(M, Fin * K))
    _, y2 = ops.cheb_forward(plan, x2, W, K)
    _, y12 = ops.cheb_forward(plan, 2 * x1 + x2, W, K)
    torch.cuda.synchronize()
    err = O.normwise_err(y12.cpu().numpy(), (2 * y1 + y2).cpu().numpy().astype(np.float64))
    assert err < 1e-5, err
