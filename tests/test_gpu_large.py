"""Large graphs on the streaming path.

  C: the reference's own 10 000-vertex cosine 16-NN graph (golden_C.npz, made
     by importing lib/graph.py): basis bit-exact to lib/graph.py::chebyshev,
     y / dx / dW within 1e-5 of the float64 truth; full layer-1 batch (N=128)
     and a Fin=32 layer-2 shape against the oracle.
     Plus the two-layer stack at the config's batch: layer 1 (Fin 1 -> 32,
     ReLU) chained into layer 2 (Fin 32 -> 32), forward and backward.
  D: the seeded Chung-Lu power-law graph (scripts/synth_graphs.py, M = 2^18,
     nnz(L~) = 4 189 524, rows up to 1 131 nnz) with Fin = Fout = 64, K = 3:
     one sample against the oracle (whose SpMM order is pinned to the
     reference's, tests/test_oracle_golden.py), batch-size-independent
     identities at N = 16 (per-sample independence, linearity), and the
     config's full per-rank workload N = 256 (the 2048 global batch over 8
     GPUs): sampled samples against the oracle and dW against a float64 GEMM.
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


@pytest.mark.parametrize("N,Fin,K,Fout", [(128, 1, 5, 32), (64, 2, 5, 16), (48, 1, 3, 8),
                                          (32, 1, 4, 40)])
def test_config_c_wide_vs_narrow_layout(dev, graph_c, N, Fin, K, Fout):
    """Config C layer 1 (Fin < 8) on the wide-column streaming layout
    (cheb_wide.hip, [M][Fin*N]; B % 128 == 0: 8 XCD column groups, else one;
    Fout % 8 == 0 and <= 32: the fused dy pass, else the row-GEMM planes)
    vs the sample-major layout (variant 'narrow'): both vs the oracle incl.
    the dx accumulation of the residual block's backward; the forward
    (basis, y) bitwise equal between the layouts."""
    from cnn_graph_amd import ops
    from cnn_graph_amd.plan import ChebPlan
    rp, ci, v, M = graph_c["Lt_rowptr"], graph_c["Lt_col"], graph_c["Lt_val"], graph_c["M"]
    rng = np.random.default_rng(3 * N + Fin)
    x = rng.random((N, M, Fin), dtype=np.float32)
    W = (rng.standard_normal((Fin * K, Fout)) * 0.1).astype(np.float32)
    dy = rng.standard_normal((N, M, Fout)).astype(np.float32)
    dx0 = rng.standard_normal((N, M, Fin)).astype(np.float32)
    out = {}
    for variant in ("auto", "narrow"):
        plan = ChebPlan(scipy.sparse.csr_matrix((v, ci, rp), shape=(M, M)), device=0, variant=variant)
        assert plan.query_path(N, Fin, K, Fout) == "stream"
        basis, y = ops.cheb_forward(plan, t(x, dev), t(W, dev), K)
        dx, dW = ops.cheb_backward(plan, t(dy, dev), basis, t(W, dev), K)
        dxa = t(dx0, dev)
        ops.cheb_backward_ex(plan, t(dy, dev), None, "none", basis, t(W, dev), K, dx=dxa,
                             dx_accumulate=True)
        torch.cuda.synchronize()
        out[variant] = [a.cpu().numpy() for a in (basis, y, dx, dW, dxa)]
    ob, oy = O.cheb_forward(x, rp, ci, v, W, K)
    odx, odW = O.cheb_backward(dy, ob, W, rp, ci, v, N, M, Fin, K)
    for variant, (basis, y, dx, dW, dxa) in out.items():
        assert np.array_equal(basis, ob), variant
        assert O.normwise_err(y, oy) < TOL, variant
        assert O.normwise_err(dx, odx) < TOL, variant
        assert O.normwise_err(dW, odW) < TOL, variant
        assert O.normwise_err(dxa, odx + dx0) < TOL, variant
    for a, b in zip(out["auto"][:2], out["narrow"][:2]):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("N,Fin,K,Fout", [(128, 1, 5, 32), (64, 2, 3, 16)])
def test_dx_only_backward_without_basis(dev, graph_c, N, Fin, K, Fout):
    """A dx-only backward (dW not wanted) may pass basis = NULL (the recurrent
    callers do): on the wide-column shapes whose dy pass also computes dW
    partials (Fin < 8, Fin*K <= 32, Fout % 8 == 0, <= 32) the basis loads are
    skipped; dx is bitwise the dx of the call that had the basis."""
    from cnn_graph_amd import ops
    from cnn_graph_amd.plan import ChebPlan
    rp, ci, v, M = graph_c["Lt_rowptr"], graph_c["Lt_col"], graph_c["Lt_val"], graph_c["M"]
    rng = np.random.default_rng(N + Fin)
    x = rng.random((N, M, Fin), dtype=np.float32)
    W = (rng.standard_normal((Fin * K, Fout)) * 0.1).astype(np.float32)
    dy = rng.standard_normal((N, M, Fout)).astype(np.float32)
    plan = ChebPlan(scipy.sparse.csr_matrix((v, ci, rp), shape=(M, M)), device=0)
    assert plan.query_path(N, Fin, K, Fout) == "stream"
    basis, _ = ops.cheb_forward(plan, t(x, dev), t(W, dev), K)
    dx_ref, _ = ops.cheb_backward(plan, t(dy, dev), basis, t(W, dev), K)
    dx, dW = ops.cheb_backward(plan, t(dy, dev), None, t(W, dev), K, need_dW=False)
    torch.cuda.synchronize()
    assert dW is None
    assert torch.equal(dx, dx_ref)
    ob, _ = O.cheb_forward(x, rp, ci, v, W, K)
    odx, _ = O.cheb_backward(dy, ob, W, rp, ci, v, N, M, Fin, K)
    assert O.normwise_err(dx.cpu().numpy(), odx) < TOL


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


@pytest.mark.timeout(600)
def test_config_c_two_layers_chained_full_batch(dev, graph_c):
    """Config C as the two-layer stack it is (BASELINE: "2 cheb layers",
    SURVEY §8d F = [32, 32]) at its batch N = 128: h = relu(cheb(x; W1)) with
    Fin 1 -> 32, y = cheb(h; W2) with Fin 32 -> 32, then the backward of both.
    Each layer is checked against the oracle on the inputs it actually got:
    layer 2's basis bit-exact on the GPU's h, every output / gradient within
    1e-5 of float64 (the ReLU mask of the backward is the GPU's h > 0)."""
    from cnn_graph_amd import ops
    rp, ci, v, M = graph_c["Lt_rowptr"], graph_c["Lt_col"], graph_c["Lt_val"], graph_c["M"]
    N, K, F1, F2 = 128, 5, 32, 32
    rng = np.random.default_rng(2048)
    x = rng.random((N, M, 1), dtype=np.float32)
    W1 = (rng.standard_normal((1 * K, F1)) * 0.1).astype(np.float32)
    W2 = (rng.standard_normal((F1 * K, F2)) * 0.1).astype(np.float32)
    dy = rng.standard_normal((N, M, F2)).astype(np.float32)
    plan = plan_of(rp, ci, v, M)
    assert plan.query_path(N, F1, K, F2) == "stream"
    b1, h = ops.cheb_forward(plan, t(x, dev), t(W1, dev), K, act="relu")
    b2, y = ops.cheb_forward(plan, h, t(W2, dev), K)
    dh, dW2 = ops.cheb_backward(plan, t(dy, dev), b2, t(W2, dev), K)
    dx, dW1, _ = ops.cheb_backward_ex(plan, dh, h, "relu", b1, t(W1, dev), K)
    torch.cuda.synchronize()
    hg = h.cpu().numpy()
    # layer 1
    ob1, oy1 = O.cheb_forward(x, rp, ci, v, W1, K)
    assert np.array_equal(b1.cpu().numpy(), ob1)
    assert O.normwise_err(hg, np.maximum(oy1, 0)) < TOL
    # layer 2 on the GPU's h
    ob2, oy2 = O.cheb_forward(hg, rp, ci, v, W2, K)
    assert np.array_equal(b2.cpu().numpy(), ob2), "layer-2 basis not bit-exact"
    assert O.normwise_err(y.cpu().numpy(), oy2) < TOL
    odh, odW2 = O.cheb_backward(dy, ob2, W2, rp, ci, v, N, M, F1, K)
    assert O.normwise_err(dh.cpu().numpy(), odh) < TOL
    assert O.normwise_err(dW2.cpu().numpy(), odW2) < TOL
    dz = np.where(hg > 0, dh.cpu().numpy().astype(np.float64), 0.0)
    odx, odW1 = O.cheb_backward(dz, ob1, W1, rp, ci, v, N, M, 1, K)
    assert O.normwise_err(dx.cpu().numpy(), odx) < TOL
    assert O.normwise_err(dW1.cpu().numpy(), odW1) < TOL


@pytest.mark.timeout(900)
def test_config_d_full_per_rank_batch(dev, graph_d):
    """Config D at its per-rank workload: N = 256 (2 048 over 8 GPUs),
    M = 2^18, Fin = Fout = 64, K = 3 -- x, dy, y, dx 17.2 GB each, the basis
    51.5 GB and one shared 51.5 GB workspace (ChebRunner; the reverse
    recurrence runs in place of dBasis), ~172 GB of the 288 GB HBM.  Samples
    0, 131 and 255: basis bit-exact, y and dx within 1e-5 of the float64
    oracle.  Every sample: y, dx and dW (a sum over all 256 samples) within
    1e-5 of an independent float64 forward / backward (`_f64_cheb_chunks`:
    torch index_add over the CSR of L~, not the product kernels and not the
    GPU's basis)."""
    from cnn_graph_amd import ops
    rp, ci, v, M = graph_d
    N, Fin, K, Fout = 256, 64, 3, 64
    FinK = Fin * K
    plan = plan_of(rp, ci, v, M)
    assert plan.query_path(N, Fin, K, Fout) == "stream"
    fb, bb = plan.workspace_bytes(N, Fin, K, Fout)
    assert max(fb, bb) <= 4 * N * M * FinK + (64 << 20)
    run = ops.ChebRunner(plan, N, Fin, K, Fout, dev)
    g = torch.Generator(device=dev)
    g.manual_seed(2017)
    x = torch.rand((N, M, Fin), device=dev, generator=g)
    W = torch.randn((FinK, Fout), device=dev, generator=g) * 0.1
    dy = torch.randn((N, M, Fout), device=dev, generator=g)
    y = run.forward(x, W)
    dx, dW = run.backward(dy, W)
    torch.cuda.synchronize()
    Wn = W.cpu().numpy()
    basis = run.basis.view(N, M, FinK)
    for n in (0, 131, 255):
        xn = x[n:n + 1].cpu().numpy()
        dyn = dy[n:n + 1].cpu().numpy()
        ob, oy = O.cheb_forward(xn, rp, ci, v, Wn, K)
        assert np.array_equal(basis[n].cpu().numpy(), ob), f"sample {n}: basis not bit-exact"
        assert O.normwise_err(y[n:n + 1].cpu().numpy(), oy) < TOL
        odx, _ = O.cheb_backward(dyn, ob, Wn, rp, ci, v, 1, M, Fin, K)
        assert O.normwise_err(dx[n:n + 1].cpu().numpy(), odx) < TOL
    del basis
    run.basis = run.ws = run.fws = run.bws = None  # 103 GB back for the float64 pass
    torch.cuda.empty_cache()
    dev_y, ref_y, dev_dx, ref_dx = 0.0, 0.0, 0.0, 0.0
    dW_ref = None
    for c, y64, dx64, dW_ref in _f64_cheb_chunks(rp, ci, v, M, x, W, dy, K, dev):
        dev_y = max(dev_y, float((y[c] - y64).abs().max()))
        ref_y = max(ref_y, float(y64.abs().max()))
        dev_dx = max(dev_dx, float((dx[c] - dx64).abs().max()))
        ref_dx = max(ref_dx, float(dx64.abs().max()))
    assert dev_y / ref_y < TOL, ("y", dev_y / ref_y)
    assert dev_dx / ref_dx < TOL, ("dx", dev_dx / ref_dx)
    assert O.normwise_err(dW.cpu().numpy(), dW_ref.cpu().numpy()) < TOL


def _f64_cheb_chunks(rp, ci, v, M, x, W, dy, K, dev, chunk=2):
    """chebyshev5 forward and backward of every sample in float64 on the GPU,
    `chunk` samples at a time, written independently of the product kernels
    (torch index_add over the CSR of L~ and L~^T; the basis layout of
    lib/graph_conv.py:170-172, column j = fin*K + k; backward = TF's autodiff
    of it: dT_k = dy W_k^T, dx by the Clenshaw recurrence over L~^T).
    Yields (sample slice, y [c, M, Fout], dx [c, M, Fin], dW so far)."""
    N, _, Fin = x.shape
    Fout = W.shape[1]
    row = torch.as_tensor(np.repeat(np.arange(M), np.diff(rp)), device=dev)
    col = torch.as_tensor(ci.astype(np.int64), device=dev)
    val = torch.as_tensor(v.astype(np.float64), device=dev)[:, None]

    def lmul(X):  # L~ X
        return torch.zeros_like(X).index_add_(0, row, val * X[col])

    def ltmul(X):  # L~^T X
        return torch.zeros_like(X).index_add_(0, col, val * X[row])

    Wk = W.double().view(Fin, K, Fout)
    dW = torch.zeros((Fin, K, Fout), dtype=torch.float64, device=dev)
    for c0 in range(0, N, chunk):
        c = slice(c0, min(c0 + chunk, N))
        nc = c.stop - c.start
        X = x[c].double().permute(1, 0, 2).reshape(M, nc * Fin)
        T = [X]
        if K > 1:
            T.append(lmul(X))
        for _ in range(2, K):
            T.append(2.0 * lmul(T[-1]) - T[-2])
        dyc = dy[c].double()
        y64 = torch.zeros((nc, M, Fout), dtype=torch.float64, device=dev)
        dB = []
        for k in range(K):
            Tk = T[k].view(M, nc, Fin)
            y64 += torch.einsum("mnf,fo->nmo", Tk, Wk[:, k])
            dW[:, k] += torch.einsum("mnf,nmo->fo", Tk, dyc)
            dB.append(torch.einsum("nmo,fo->mnf", dyc, Wk[:, k]).reshape(M, nc * Fin))
        del T
        b1 = torch.zeros_like(X)
        b2 = torch.zeros_like(X)
        for k in range(K - 1, 0, -1):
            b1, b2 = dB[k] + 2.0 * ltmul(b1) - b2, b1
        dx64 = dB[0] + ltmul(b1) - b2
        yield c, y64, dx64.view(M, nc, Fin).permute(1, 0, 2), dW.view(Fin * K, Fout)


@pytest.mark.parametrize("which", ["C", "D"])
def test_gemm_x3_streaming_vs_oracle(dev, cg_opts, graph_c, graph_d, which):
    """CG_OPT_GEMM_X3 = 1: the streaming path's row GEMMs (y = basis W, dBasis
    = dy W^T) on the split-bf16 matrix pipe: basis still bit-exact, y / dx / dW
    within 1e-5 of the float64 oracle (config C at its Fin = 32 layer-2 shape,
    N = 4; config D one sample, Fin = Fout = 64, K = 3)."""
    from cnn_graph_amd import ops
    if which == "C":
        rp, ci, v, M = graph_c["Lt_rowptr"], graph_c["Lt_col"], graph_c["Lt_val"], graph_c["M"]
        N, Fin, K, Fout = 4, 32, 5, 32
    else:
        rp, ci, v, M = graph_d
        N, Fin, K, Fout = 1, 64, 3, 64
    rng = np.random.default_rng(23)
    x = rng.random((N, M, Fin), dtype=np.float32)
    W = (rng.standard_normal((Fin * K, Fout)) * 0.1).astype(np.float32)
    dy = rng.standard_normal((N, M, Fout)).astype(np.float32)
    plan = plan_of(rp, ci, v, M)
    assert plan.query_path(N, Fin, K, Fout) == "stream"
    cg_opts("gemm_x3", 1)
    basis, y = ops.cheb_forward(plan, t(x, dev), t(W, dev), K)
    dx, dW = ops.cheb_backward(plan, t(dy, dev), basis, t(W, dev), K)
    torch.cuda.synchronize()
    ob, oy = O.cheb_forward(x, rp, ci, v, W, K)
    assert np.array_equal(basis.cpu().numpy().reshape(ob.shape), ob)
    assert O.normwise_err(y.cpu().numpy(), oy) < TOL
    odx, odW = O.cheb_backward(dy, ob, W, rp, ci, v, N, M, Fin, K)
    assert O.normwise_err(dx.cpu().numpy(), odx) < TOL
    assert O.normwise_err(dW.cpu().numpy(), odW) < TOL
