"""Basis layouts other than the reference's rows layout.

Orders basis layout (CG_BASIS_ORDERS, [N][Fin*K][Mb]): the fast forward
stores each Chebyshev order pair during the recurrence and the fused-dW fast
backward reads the planes back.  Bar: basis (re-laid to rows), y and dx
BITWISE equal to the rows layout (lib/graph_conv.py:172) and the basis bitwise
equal to the reference-generated golden basis; padding rows zero; dW (which
sums its per-wave row chunks in another grouping) within 1e-6 normwise of the
rows-layout dW and 1e-5 of the golden/oracle dW; Adam on top agrees.
Planes layout (CG_BASIS_PLANES, [K][N*M][Fin]): see the section at the end."""
import numpy as np
import pytest
import scipy.sparse

from conftest import case, load_golden
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


def _plan(c):
    from cnn_graph_amd.plan import ChebPlan
    M = c["M"]
    Lt = scipy.sparse.csr_matrix((c["Lt_val"], c["Lt_col"], c["Lt_rowptr"]), shape=(M, M))
    return ChebPlan(Lt, device=0, path="resident")


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(dev)


def _pair(plan, N, Fin, K, Fout, dev, x, W, dy):
    from cnn_graph_amd import ops
    rr = ops.ChebRunner(plan, N, Fin, K, Fout, dev, basis_layout="rows")
    ro = ops.ChebRunner(plan, N, Fin, K, Fout, dev, basis_layout="orders")
    assert ro.basis_layout == "orders"
    for r in (rr, ro):
        r.forward(x, W)
        r.backward(dy, W)
    torch.cuda.synchronize()
    return rr, ro


def _check_pair(rr, ro, M):
    assert torch.equal(ro.basis_rows(), rr.basis), "orders basis differs from the rows basis"
    assert int(torch.count_nonzero(ro.basis[:, :, M:])) == 0, "padding rows not zero"
    assert torch.equal(ro.y, rr.y)
    assert torch.equal(ro.dx, rr.dx)
    assert O.normwise_err(ro.dW.cpu().double().numpy(), rr.dW.cpu().double().numpy()) < 1e-6


@pytest.mark.parametrize("name", ["golden_B.npz", "golden_E.npz"])
def test_orders_layout_golden(dev, name):
    c = case(load_golden(name))
    M, N, Fin, K, Fout = c["M"], c["N"], c["Fin"], c["K"], c["Fout"]
    plan = _plan(c)
    Mb = (M + 31) // 32 * 32
    assert plan.basis_elems(N, Fin, K, Fout, "orders") == N * Fin * K * Mb
    assert plan.basis_elems(N, Fin, K, Fout, "rows") == N * M * Fin * K
    rr, ro = _pair(plan, N, Fin, K, Fout, dev, _t(c["x"], dev), _t(c["W"], dev), _t(c["dy"], dev))
    _check_pair(rr, ro, M)
    assert np.array_equal(ro.basis_rows().cpu().numpy(), c["basis"].astype(np.float32))
    assert O.normwise_err(ro.y.cpu().double().numpy(), c["y_ref"]) < 1e-5
    assert O.normwise_err(ro.dx.cpu().double().numpy(), c["dx_ref"]) < 1e-5
    assert O.normwise_err(ro.dW.cpu().double().numpy(), c["dW_ref"]) < 1e-5


@pytest.mark.parametrize("N,Fin,K", [(256, 1, 25), (96, 2, 8), (64, 2, 3), (40, 1, 2), (33, 1, 1)])
def test_orders_layout_config_b_shapes(dev, N, Fin, K):
    """Config B's graph at the bench batch (N = 256) and at other Fin/K/N,
    including K = 1 (no recurrence) and K = 2 (one half-empty pair)."""
    c = case(load_golden("golden_B.npz"))
    M, Fout = c["M"], 32
    plan = _plan(c)
    g = torch.Generator().manual_seed(1000 + N + Fin + K)
    x = torch.rand((N, M, Fin), generator=g).to(dev)
    W = (torch.randn((Fin * K, Fout), generator=g) * 0.1).to(dev)
    dy = torch.randn((N, M, Fout), generator=g).to(dev)
    rr, ro = _pair(plan, N, Fin, K, Fout, dev, x, W, dy)
    _check_pair(rr, ro, M)
    # against the oracle (basis bit-exact, dW / dx to 1e-5) where it is quick
    if N <= 64:
        rp, ci, va = c["Lt_rowptr"], c["Lt_col"], c["Lt_val"]
        xs, Ws, dys = (t.cpu().numpy() for t in (x, W, dy))
        basis, _ = O.cheb_forward(xs, rp, ci, va, Ws, K)
        assert np.array_equal(ro.basis_rows().cpu().numpy(), basis)
        dx64, dW64 = O.cheb_backward(dys, basis, Ws, rp, ci, va, N, M, Fin, K)
        assert O.normwise_err(ro.dW.cpu().double().numpy(), dW64) < 1e-5
        assert O.normwise_err(ro.dx.cpu().double().numpy(), dx64) < 1e-5


def test_orders_layout_adam(dev):
    c = case(load_golden("golden_B.npz"))
    M, N, Fin, K, Fout = c["M"], c["N"], c["Fin"], c["K"], c["Fout"]
    from cnn_graph_amd import ops
    plan = _plan(c)
    x, dy, W0 = _t(c["x"], dev), _t(c["dy"], dev), _t(c["W"], dev)
    rr = ops.ChebRunner(plan, N, Fin, K, Fout, dev, basis_layout="rows")
    ro = ops.ChebRunner(plan, N, Fin, K, Fout, dev, basis_layout="orders")
    Wr, Wo = W0.clone(), W0.clone()
    mr, vr, mo, vo = (torch.zeros_like(W0) for _ in range(4))
    for step in (1, 2, 3):
        rr.forward(x, Wr)
        ro.forward(x, Wo)
        rr.backward_adam(dy, Wr, mr, vr, step)
        ro.backward_adam(dy, Wo, mo, vo, step)
        torch.cuda.synchronize()
        if step == 1:  # later steps start from W that differ by dW's rounding
            assert torch.equal(ro.dx, rr.dx), "dx differs at equal W"
        else:
            assert O.normwise_err(ro.dx.cpu().double().numpy(), rr.dx.cpu().double().numpy()) < 1e-5
        assert O.normwise_err(Wo.cpu().double().numpy(), Wr.cpu().double().numpy()) < 1e-6


def test_orders_layout_unsupported(dev):
    from cnn_graph_amd import _lib, ops
    c = case(load_golden("golden_B.npz"))
    M = c["M"]
    plan = _plan(c)
    # Fout = 64: no fused dW in the fast backward -> rows only
    assert plan.basis_elems(8, 1, 25, 64, "orders") is None
    with pytest.raises(ValueError):
        ops.ChebRunner(plan, 8, 1, 25, 64, dev, basis_layout="orders")
    with pytest.raises(ValueError):
        ops.ChebRunner(plan, 8, 1, 25, 32, dev, basis_layout="auto")
    # config A's graph has a 21-nonzero row: classic resident kernels, rows only
    a = case(load_golden("golden_A.npz"))
    assert _plan(a).basis_elems(a["N"], 1, a["K"], a["Fout"], "orders") is None
    # the streaming path never takes it
    from cnn_graph_amd.plan import ChebPlan
    Lt = scipy.sparse.csr_matrix((c["Lt_val"], c["Lt_col"], c["Lt_rowptr"]), shape=(M, M))
    assert ChebPlan(Lt, device=0, path="stream").basis_elems(8, 1, 25, 32, "orders") is None
    # dW is fused into the dx pass: dW without dx is refused
    ro = ops.ChebRunner(plan, 8, 1, 25, 32, dev, basis_layout="orders")
    x = torch.rand((8, M, 1), device=dev)
    W = torch.randn((25, 32), device=dev)
    ro.forward(x, W)
    with pytest.raises(_lib.CGError):
        ro.backward(torch.randn((8, M, 32), device=dev), W, need_dx=False)



# ---- planes layout (CG_BASIS_PLANES, [K][N*M][Fin]) ---------------------------------
# The streaming path's layout for the ResGNN hidden layers: each Chebyshev step
# writes T_k as its own plane (plane 0 = x), the rows-layout assembly pass
# disappears, the row GEMM and the dW slabs read the planes.  Bar: basis
# (re-laid to rows) and dx BITWISE equal to the rows layout, dW bitwise too
# (each dW element sums the same rows in the same order), y within 1e-5 of the
# float64 oracle (its inner dimension is summed in another order).
@pytest.mark.parametrize("N,Fin,K,Fout", [(4, 32, 6, 32), (5, 32, 20, 32), (3, 16, 4, 40),
                                          (2, 64, 3, 64)])
def test_planes_layout_vs_rows(dev, N, Fin, K, Fout):
    from cnn_graph_amd import ops
    from cnn_graph_amd.plan import ChebPlan
    c = case(load_golden("golden_B.npz"))
    M = c["M"]
    Lt = scipy.sparse.csr_matrix((c["Lt_val"], c["Lt_col"], c["Lt_rowptr"]), shape=(M, M))
    plan = ChebPlan(Lt, device=0, path="stream")
    rng = np.random.default_rng(N * 1000 + Fin + K)
    x = rng.standard_normal((N, M, Fin)).astype(np.float32)
    W = (rng.standard_normal((Fin * K, Fout)) * 0.1).astype(np.float32)
    dy = rng.standard_normal((N, M, Fout)).astype(np.float32)
    res = rng.standard_normal((N, M, Fout)).astype(np.float32)
    rr = ops.ChebRunner(plan, N, Fin, K, Fout, dev, basis_layout="rows")
    rp = ops.ChebRunner(plan, N, Fin, K, Fout, dev, basis_layout="planes")
    assert tuple(rp.basis.shape) == (K, N * M, Fin)
    xt, Wt, dyt = _t(x, dev), _t(W, dev), _t(dy, dev)
    for r in (rr, rp):
        r.forward(xt, Wt)
        r.backward(dyt, Wt)
    torch.cuda.synchronize()
    assert torch.equal(rp.basis_rows(), rr.basis), "planes basis differs from the rows basis"
    assert torch.equal(rp.dx, rr.dx)
    assert torch.equal(rp.dW, rr.dW)
    b64 = rr.basis.cpu().numpy().astype(np.float64)
    y64 = (b64 @ W.astype(np.float64)).reshape(N, M, Fout)
    assert O.normwise_err(rp.y.cpu().numpy(), y64) < 1e-5
    # the residual + ReLU epilogue of the planes row GEMM (cg_cheb_forward_layout)
    from cnn_graph_amd import _lib
    y2 = torch.empty((N, M, Fout), device=dev)
    _lib.check("cg_cheb_forward_layout", _lib.lib().cg_cheb_forward_layout(
        plan.handle, N, Fin, K, Fout, xt.data_ptr(), Wt.data_ptr(), _t(res, dev).data_ptr(),
        _lib.CG_ACT_RELU, _lib.CG_BASIS_PLANES, rp.basis.data_ptr(), y2.data_ptr(),
        rp.ws.data_ptr(), rp.fwd_bytes, torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    assert O.normwise_err(y2.cpu().numpy(), np.maximum(y64 + res, 0)) < 1e-5


def test_planes_layout_unsupported(dev):
    """Resident shapes, Fin not a multiple of 16 and K = 1 refuse the planes layout."""
    from cnn_graph_amd.plan import ChebPlan
    c = case(load_golden("golden_B.npz"))
    M = c["M"]
    Lt = scipy.sparse.csr_matrix((c["Lt_val"], c["Lt_col"], c["Lt_rowptr"]), shape=(M, M))
    auto = ChebPlan(Lt, device=0, path="auto")
    stream = ChebPlan(Lt, device=0, path="stream")
    assert auto.basis_elems(8, 1, 25, 32, "planes") is None   # fast resident path
    assert stream.basis_elems(8, 8, 5, 32, "planes") is None  # Fin % 16 != 0
    assert stream.basis_elems(8, 32, 1, 32, "planes") is None  # K = 1
    assert stream.basis_elems(8, 32, 5, 32, "planes") == 8 * M * 32 * 5


def test_autograd_uses_planes_with_rows_gradients(dev):
    """ops.cheb_conv (the GraphConv.chebyshev5 autograd path) keeps its saved
    basis in the planes layout on a Fin = 32 streaming shape: its dx and dW are
    bitwise the explicit rows-layout backward's, y within 1e-5 of float64."""
    from cnn_graph_amd import ops
    from cnn_graph_amd.plan import ChebPlan
    c = case(load_golden("golden_B.npz"))
    M = c["M"]
    Lt = scipy.sparse.csr_matrix((c["Lt_val"], c["Lt_col"], c["Lt_rowptr"]), shape=(M, M))
    plan = ChebPlan(Lt, device=0, path="stream")
    N, Fin, K, Fout = 3, 32, 5, 32
    assert ops.basis_layout_for(plan, N, Fin, K, Fout) == "planes"
    rng = np.random.default_rng(9)
    x = _t(rng.standard_normal((N, M, Fin)), dev).requires_grad_(True)
    W = _t(rng.standard_normal((Fin * K, Fout)) * 0.1, dev).requires_grad_(True)
    dy = _t(rng.standard_normal((N, M, Fout)), dev)
    y = ops.cheb_conv(x, W, plan, K)
    y.backward(dy)
    basis, y_rows = ops.cheb_forward(plan, x.detach(), W.detach(), K)
    dx_r, dW_r = ops.cheb_backward(plan, dy, basis, W.detach(), K)
    torch.cuda.synchronize()
    assert torch.equal(x.grad, dx_r) and torch.equal(W.grad, dW_r)
    y64 = (basis.cpu().numpy().astype(np.float64) @ W.detach().cpu().numpy().astype(np.float64))
    assert O.normwise_err(y.detach().cpu().numpy().reshape(N * M, Fout), y64) < 1e-5


def test_autograd_planes_basis_after_path_change(dev):
    """The plan's path is changed between an autograd forward (streaming,
    planes-layout basis saved) and its backward (now resident, where the
    planes layout does not apply): the backward re-lays the saved basis as
    rows and matches the streaming rows-layout gradients."""
    from cnn_graph_amd import ops
    from cnn_graph_amd.plan import ChebPlan
    c = case(load_golden("golden_A.npz"))
    M = c["M"]
    Lt = scipy.sparse.csr_matrix((c["Lt_val"], c["Lt_col"], c["Lt_rowptr"]), shape=(M, M))
    plan = ChebPlan(Lt, device=0, path="stream")
    N, Fin, K, Fout = 4, 16, 3, 16
    assert ops.basis_layout_for(plan, N, Fin, K, Fout) == "planes"
    rng = np.random.default_rng(19)
    x = _t(rng.standard_normal((N, M, Fin)), dev).requires_grad_(True)
    W = _t(rng.standard_normal((Fin * K, Fout)) * 0.1, dev).requires_grad_(True)
    dy = _t(rng.standard_normal((N, M, Fout)), dev)
    basis, _ = ops.cheb_forward(plan, x.detach(), W.detach(), K)
    dx_r, dW_r = ops.cheb_backward(plan, dy, basis, W.detach(), K)
    y = ops.cheb_conv(x, W, plan, K)
    plan.set_path("auto")
    assert plan.query_path(N, Fin, K, Fout) == "resident"
    assert ops.basis_layout_for(plan, N, Fin, K, Fout) == "rows"
    y.backward(dy)
    torch.cuda.synchronize()
    assert O.normwise_err(x.grad.cpu().numpy(), dx_r.cpu().numpy().astype(np.float64)) < 1e-5
    assert O.normwise_err(W.grad.cpu().numpy(), dW_r.cpu().numpy().astype(np.float64)) < 1e-5


def test_planes_layout_skewed_graph(dev):
    """Planes vs rows on a hub-and-spoke graph whose row lengths are skewed
    enough for the degree-sorted row order (max row > 2 * mean + 8): the
    steps visit rows in that order and write their planes in natural order."""
    from cnn_graph_amd import ops
    from cnn_graph_amd.plan import ChebPlan
    rng = np.random.default_rng(5)
    M, hubs = 1500, 6
    rows, cols = [], []
    for v in range(M):                       # a ring
        rows += [v, (v + 1) % M]
        cols += [(v + 1) % M, v]
    for hbv in range(hubs):                  # hubs linked to ~150 random vertices each
        nb = rng.choice(np.arange(hubs, M), size=150, replace=False)
        rows += [hbv] * len(nb) + list(nb)
        cols += list(nb) + [hbv] * len(nb)
    A = scipy.sparse.csr_matrix((np.ones(len(rows), np.float32), (rows, cols)), shape=(M, M))
    A.sum_duplicates()
    A.data[:] = 1.0
    d = np.asarray(A.sum(axis=1)).ravel()
    Dm = scipy.sparse.diags((1.0 / np.sqrt(d)).astype(np.float32))
    Lt = (-(Dm @ A @ Dm)).astype(np.float32).tocsr()   # L~ = L - I for lmax = 2
    Lt.sort_indices()
    lens = np.diff(Lt.indptr)
    assert lens.max() > 2 * (Lt.nnz // M) + 8, "graph not skewed enough for the sorted row order"
    plan = ChebPlan(Lt, device=0, path="stream")
    N, Fin, K, Fout = 2, 16, 4, 16
    x = _t(rng.standard_normal((N, M, Fin)), dev)
    W = _t(rng.standard_normal((Fin * K, Fout)) * 0.1, dev)
    dy = _t(rng.standard_normal((N, M, Fout)), dev)
    rr = ops.ChebRunner(plan, N, Fin, K, Fout, dev, basis_layout="rows")
    rp = ops.ChebRunner(plan, N, Fin, K, Fout, dev, basis_layout="planes")
    for r in (rr, rp):
        r.forward(x, W)
        r.backward(dy, W)
    torch.cuda.synchronize()
    assert torch.equal(rp.basis_rows(), rr.basis)
    assert torch.equal(rp.dx, rr.dx) and torch.equal(rp.dW, rr.dW)
    assert O.normwise_err(rp.y.cpu().numpy(), rr.y.cpu().numpy().astype(np.float64)) < 1e-5
    # and the basis against the float64 recurrence of the oracle
    xb = x.cpu().numpy().astype(np.float64)
    T = [xb, np.stack([Lt @ xb[n] for n in range(N)])]
    for _ in range(2, K):
        T.append(np.stack([2 * (Lt @ T[-1][n]) for n in range(N)]) - T[-2])
    ref = np.stack(T, axis=-1).reshape(N * M, Fin * K)  # column fin*K + k
    assert O.normwise_err(rr.basis.cpu().numpy(), ref) < 1e-5


@pytest.mark.parametrize("variant,gname,N,Fin,K,Fout", [("steps", "golden_B.npz", 3, 32, 5, 32),
                                                        ("auto", "golden_B.npz", 3, 32, 6, 32),
                                                        ("auto", "golden_C.npz", 2, 32, 5, 32)])
def test_planes_input_in_plane0_bitwise(dev, variant, gname, N, Fin, K, Fout):
    """The planes layout with x placed in plane 0 of the basis (x == basis:
    cg_cheb_forward_layout reads T_0 in place, no copy; the channel-group
    kernels skip their plane-0 write) against x in its own buffer: basis, y,
    dx and dW bitwise equal -- on the streaming steps (variant 'steps', and
    config C's 10 000-vertex graph) and on the channel-group kernels."""
    from cnn_graph_amd import ops
    from cnn_graph_amd.plan import ChebPlan
    c = case(load_golden(gname))
    M = c["M"]
    Lt = scipy.sparse.csr_matrix((c["Lt_val"], c["Lt_col"], c["Lt_rowptr"]), shape=(M, M))
    plan = ChebPlan(Lt, device=0, path="stream", variant=variant)
    rng = np.random.default_rng(N + Fin + K + M)
    xt = _t(rng.standard_normal((N, M, Fin)), dev)
    Wt = _t(rng.standard_normal((Fin * K, Fout)) * 0.1, dev)
    dyt = _t(rng.standard_normal((N, M, Fout)), dev)
    ra = ops.ChebRunner(plan, N, Fin, K, Fout, dev, basis_layout="planes")
    rb = ops.ChebRunner(plan, N, Fin, K, Fout, dev, basis_layout="planes")
    assert ra.input_plane().data_ptr() == ra.basis.data_ptr()
    ra.forward(xt, Wt)
    x0 = rb.input_plane()
    x0.copy_(xt)
    rb.forward(x0, Wt)
    for r in (ra, rb):
        r.backward(dyt, Wt)
    torch.cuda.synchronize()
    assert torch.equal(x0, xt)  # T_0 read in place, never rewritten
    assert torch.equal(ra.basis, rb.basis)
    assert torch.equal(ra.y, rb.y)
    assert torch.equal(ra.dx, rb.dx)
    assert torch.equal(ra.dW, rb.dW)


@pytest.mark.parametrize("layout", ["orders", "rows"])
def test_fast_backward_x3_vs_f32(dev, cg_opts, layout):
    """The fast backward's split-bf16 dBasis (and, orders layout, fused dW:
    cheb_bwd_fast<FV, 3>) against its f32-MFMA form (CG_OPT_GEMM_X3 = 0) on
    config B's shape at the bench batch: dx and dW agree to f32 rounding
    (1e-6 normwise) and both sit within 1e-5 of the float64 oracle on a
    64-sample slice; the forward is untouched (basis and y bitwise)."""
    from cnn_graph_amd import ops
    c = case(load_golden("golden_B.npz"))
    M, N, Fin, K, Fout = c["M"], 256, 1, 25, 32
    plan = _plan(c)
    g = torch.Generator().manual_seed(77)
    x = torch.rand((N, M, Fin), generator=g).to(dev)
    W = (torch.randn((Fin * K, Fout), generator=g) * 0.1).to(dev)
    dy = torch.randn((N, M, Fout), generator=g).to(dev)
    out = {}
    for x3 in (0, 1):
        cg_opts("gemm_x3", x3)
        r = ops.ChebRunner(plan, N, Fin, K, Fout, dev, basis_layout=layout)
        r.forward(x, W)
        r.backward(dy, W)
        torch.cuda.synchronize()
        out[x3] = (r.basis.clone(), r.y.clone(), r.dx.clone(), r.dW.clone())
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])
    for i in (2, 3):
        err = O.normwise_err(out[1][i].cpu().double().numpy(), out[0][i].cpu().double().numpy())
        assert err < 1e-6, (i, err)
    rp, ci, va = c["Lt_rowptr"], c["Lt_col"], c["Lt_val"]
    n = 64
    xs, Ws, dys = x[:n].cpu().numpy(), W.cpu().numpy(), dy[:n].cpu().numpy()
    basis, _ = O.cheb_forward(xs, rp, ci, va, Ws, K)
    dx64, _ = O.cheb_backward(dys, basis, Ws, rp, ci, va, n, M, Fin, K)
    basis_all, _ = O.cheb_forward(x.cpu().numpy(), rp, ci, va, Ws, K)
    _, dW64 = O.cheb_backward(dy.cpu().numpy(), basis_all, Ws, rp, ci, va, N, M, Fin, K)
    for x3 in (0, 1):
        assert O.normwise_err(out[x3][2][:n].cpu().double().numpy(), dx64) < 1e-5
        assert O.normwise_err(out[x3][3].cpu().double().numpy(), dW64) < 1e-5
