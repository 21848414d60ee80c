"""Parity of the HIP path (through the C ABI) with the oracle and the golden
fixtures.  Bars: the Chebyshev basis is BIT-EXACT to the reference's fp32
recurrence (lib/graph.py::chebyshev); y / dx / dW within 1e-5
max-abs-normalised of the float64 truth; pooling values and indices exact."""
import os

import numpy as np
import pytest
import scipy.sparse

from conftest import CASES, CASE_IDS, case, load_golden
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


# Kernel variants of the resident path (cg_plan_set_variant, per plan):
# "fast" = cheb_fast.hip with the fused dW (default), "fast_nofuse" = fast
# kernels + the separate dW GEMM, "classic" = cheb_resident.hip.
VARIANTS = {"fast": "auto", "fast_nofuse": "unfused_dw", "classic": "classic"}


@pytest.fixture(params=list(VARIANTS))
def variant(request, dev):
    return VARIANTS[request.param]


def make_plan(c, path, variant="auto"):
    from cnn_graph_amd.plan import ChebPlan
    M = c["M"]
    Lt = scipy.sparse.csr_matrix((c["Lt_val"], c["Lt_col"], c["Lt_rowptr"]), shape=(M, M))
    return ChebPlan(Lt, device=0, path=path, variant=variant)


def t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def test_native_library_is_the_in_tree_build(dev):
    from cnn_graph_amd import _lib
    assert os.path.dirname(_lib.LIB_PATH).endswith("cnn_graph_amd")
    with open("/proc/self/maps") as f:
        assert any("libcheb_mi355.so" in line for line in f)


@pytest.mark.parametrize("fname,prefix", CASES, ids=CASE_IDS)
def test_resident_variants_golden(dev, variant, fname, prefix):
    test_forward_backward_golden(dev, fname, prefix, "resident", variant)


@pytest.mark.parametrize("fin", [1, 2, 4])
def test_fast_path_fin_widths_vs_oracle(dev, variant, fin):
    """Fin in {1, 2, 4} (record-vector gathers) on the MNIST graph vs the oracle."""
    from cnn_graph_amd import ops
    g = load_golden("golden_B.npz")
    c = case(g)
    rng = np.random.default_rng(7 + fin)
    N, K, Fout = 6, 7, 24
    x = rng.random((N, c["M"], fin), dtype=np.float32)
    W = (rng.standard_normal((fin * K, Fout)) * 0.1).astype(np.float32)
    dy = rng.standard_normal((N, c["M"], Fout)).astype(np.float32)
    plan = make_plan(c, "resident", variant)
    basis, y = ops.cheb_forward(plan, t(x, dev), t(W, dev), K)
    dx, dW = ops.cheb_backward(plan, t(dy, dev), basis, t(W, dev), K)
    torch.cuda.synchronize()
    ob, oy = O.cheb_forward(x, c["Lt_rowptr"], c["Lt_col"], c["Lt_val"], W, K)
    assert np.array_equal(basis.cpu().numpy(), ob)
    assert O.normwise_err(y.cpu().numpy(), oy) < TOL
    odx, odW = O.cheb_backward(dy, ob, W, c["Lt_rowptr"], c["Lt_col"], c["Lt_val"], N, c["M"], fin, K)
    assert O.normwise_err(dx.cpu().numpy(), odx) < TOL
    assert O.normwise_err(dW.cpu().numpy(), odW) < TOL


@pytest.mark.parametrize("path", ["resident", "stream"])
@pytest.mark.parametrize("fname,prefix", CASES, ids=CASE_IDS)
def test_forward_backward_golden(dev, fname, prefix, path, variant="auto"):
    from cnn_graph_amd import ops
    c = case(load_golden(fname), prefix)
    plan = make_plan(c, path, variant)
    assert plan.query_path(c["N"], c["Fin"], c["K"], c["Fout"]) == path
    x, W, dy = t(c["x"], dev), t(c["W"], dev), t(c["dy"], dev)
    basis, y = ops.cheb_forward(plan, x, W, c["K"])
    torch.cuda.synchronize()
    assert np.array_equal(basis.cpu().numpy(), c["basis"]), "basis not bit-exact"
    assert O.normwise_err(y.cpu().numpy(), c["y_ref"]) < TOL
    dx, dW = ops.cheb_backward(plan, dy, basis, W, c["K"])
    torch.cuda.synchronize()
    assert O.normwise_err(dx.cpu().numpy(), c["dx_ref"]) < TOL
    assert O.normwise_err(dW.cpu().numpy(), c["dW_ref"]) < TOL


@pytest.mark.parametrize("path", ["resident", "stream", "classic"])
def test_config_b_full_batch_vs_oracle(dev, path):
    """BASELINE config B at full size (N=256, M=976, K=25, Fout=32)."""
    from cnn_graph_amd import ops
    g = load_golden("golden_B.npz")
    c = case(g)
    rng = np.random.default_rng(99)
    N = 256
    x = rng.random((N, c["M"], 1), dtype=np.float32)
    x[:, g["fake_rows"], :] = 0
    W = c["W"]
    dy = rng.standard_normal((N, c["M"], c["Fout"])).astype(np.float32)
    plan = make_plan(c, "resident" if path == "classic" else path,
                     "classic" if path == "classic" else "auto")
    basis, y = ops.cheb_forward(plan, t(x, dev), t(W, dev), c["K"])
    dx, dW = ops.cheb_backward(plan, t(dy, dev), basis, t(W, dev), c["K"])
    torch.cuda.synchronize()
    ob, oy = O.cheb_forward(x, c["Lt_rowptr"], c["Lt_col"], c["Lt_val"], W, c["K"])
    assert np.array_equal(basis.cpu().numpy(), ob)
    assert O.normwise_err(y.cpu().numpy(), oy) < TOL
    odx, odW = O.cheb_backward(dy, ob, W, c["Lt_rowptr"], c["Lt_col"], c["Lt_val"], N, c["M"], 1, c["K"])
    assert O.normwise_err(dx.cpu().numpy(), odx) < TOL
    assert O.normwise_err(dW.cpu().numpy(), odW) < TOL


def test_resident_and_stream_agree_and_are_deterministic(dev):
    from cnn_graph_amd import ops
    c = case(load_golden("golden_E.npz"))
    outs = []
    for path in ("resident", "resident", "stream"):
        plan = make_plan(c, path)
        x, W, dy = t(c["x"], dev), t(c["W"], dev), t(c["dy"], dev)
        basis, y = ops.cheb_forward(plan, x, W, c["K"])
        dx, dW = ops.cheb_backward(plan, dy, basis, W, c["K"])
        outs.append([a.cpu().numpy() for a in (basis, y, dx, dW)])
    for a, b in zip(outs[0], outs[1]):
        assert np.array_equal(a, b), "resident path not bitwise reproducible"
    assert np.array_equal(outs[0][0], outs[2][0])
    for a, b in zip(outs[0][1:], outs[2][1:]):
        assert O.normwise_err(a, b) < TOL


def test_basis_only_forward(dev):
    """y = NULL -> chebyshev2 / lib/graph.py::chebyshev analogue."""
    from cnn_graph_amd import ops
    c = case(load_golden("golden_A.npz"))
    plan = make_plan(c, "auto")
    basis, y = ops.cheb_forward(plan, t(c["x"], dev), None, c["K"])
    assert y is None
    assert np.array_equal(basis.cpu().numpy(), c["basis"])


def test_autograd_graphconv_chebyshev5(dev):
    """The drop-in GraphConv.chebyshev5 through torch autograd."""
    from cnn_graph_amd.graph_conv import GraphConv
    g = load_golden("golden_A.npz")
    c = case(g)
    L = scipy.sparse.csr_matrix((g["L_data"], g["L_indices"], g["L_indptr"]), shape=tuple(g["L_shape"]))
    model = GraphConv(filter="chebyshev5", device=dev)
    with model.variable_scope("conv1"):
        x = t(c["x"], dev).requires_grad_(True)
        W = model._weight_variable([c["K"], c["Fout"]], regularization=False)
        with torch.no_grad():
            W.copy_(t(c["W"], dev))
        y = model.filter(x, L, c["Fout"], c["K"])
    y.backward(t(c["dy"], dev))
    assert O.normwise_err(y.detach().cpu().numpy(), c["y_ref"]) < TOL
    assert O.normwise_err(x.grad.cpu().numpy(), c["dx_ref"]) < TOL
    assert O.normwise_err(W.grad.cpu().numpy(), c["dW_ref"]) < TOL
    assert list(model.weights) == ["conv1/weights"]


def test_maxpool_avgpool_vs_oracle(dev):
    from cnn_graph_amd import ops
    x = load_golden("golden_misc.npz")["pool_x"]
    for p in (2, 4, 8):
        xt = t(x, dev).requires_grad_(True)
        y, arg = ops.mpool1_with_argmax(xt, p)
        oy, oarg = O.mpool1_forward(x, p)
        assert np.array_equal(y.detach().cpu().numpy(), oy)
        assert np.array_equal(arg.cpu().numpy(), oarg)
        dy = np.random.default_rng(p).standard_normal(oy.shape).astype(np.float32)
        y.backward(t(dy, dev))
        assert np.array_equal(xt.grad.cpu().numpy(), O.mpool1_backward(dy, oarg, x.shape[1]))
        xa = t(x, dev).requires_grad_(True)
        ya = ops.apool1(xa, p)
        np.testing.assert_allclose(ya.detach().cpu().numpy(), O.apool1_forward(x, p), rtol=1e-6)
        ya.sum().backward()
        np.testing.assert_allclose(xa.grad.cpu().numpy(), np.full(x.shape, 1.0 / p, np.float32))


def test_perm_data_vs_reference(dev):
    from cnn_graph_amd import ops
    g = load_golden("golden_B.npz")
    out = ops.perm_data(t(g["pdata_in"], dev), g["perm0"])
    assert np.array_equal(out.cpu().numpy(), g["pdata_out"].astype(np.float32))
    x3 = np.random.default_rng(1).random((3, 784, 5), dtype=np.float32)
    out3 = ops.perm_data(t(x3, dev), g["perm0"])
    assert np.array_equal(out3.cpu().numpy(), O.perm_data(x3, g["perm0"]))


def test_adam_vs_oracle(dev):
    from cnn_graph_amd import ops
    rng = np.random.default_rng(4)
    p = rng.standard_normal(800).astype(np.float32)
    m = np.zeros(800, np.float32)
    v = np.zeros(800, np.float32)
    P, Mt, Vt = t(p, dev), t(m, dev), t(v, dev)
    ref = (p.astype(np.float64), m.astype(np.float64), v.astype(np.float64))
    for step in range(1, 6):
        gr = rng.standard_normal(800).astype(np.float32)
        ops.adam_update(P, t(gr * 2, dev), Mt, Vt, step, lr=0.01, grad_scale=0.5)
        ref = O.adam_step(*ref[:1], gr.astype(np.float64), ref[1], ref[2], step, lr=0.01)
    np.testing.assert_allclose(P.cpu().numpy(), ref[0], rtol=1e-5, atol=1e-6)


def test_bad_shapes_raise(dev):
    from cnn_graph_amd import ops, _lib
    c = case(load_golden("golden_A.npz"))
    plan = make_plan(c, "auto")
    with pytest.raises(ValueError):
        ops.cheb_forward(plan, torch.zeros((2, c["M"] + 1, 1), device=dev), t(c["W"], dev), c["K"])
    with pytest.raises(ValueError):
        ops.cheb_forward(plan, torch.zeros((2, c["M"], 1)), None, c["K"])  # CPU tensor: no fallback
    big = make_plan(c, "resident")
    with pytest.raises(_lib.CGError):
        ops.cheb_forward(big, torch.zeros((1, c["M"], 4096), device=dev), None, 40)


def test_rccl_comm_single_rank_allreduce(dev):
    """cg_comm_unique_id / cg_comm_init / cg_allreduce_sum_f32 / cg_comm_destroy
    on a real GPU (1-rank communicator: the sum is the identity)."""
    from cnn_graph_amd.dist import RcclComm
    comm = RcclComm(0)
    assert comm.world == 1
    a = torch.arange(800, device=dev, dtype=torch.float32) * 0.5
    ref = a.clone()
    comm.allreduce_sum_(a)
    torch.cuda.synchronize()
    assert torch.equal(a, ref)
    comm.close()


@pytest.mark.parametrize("layout,N,Fin,K,Fout,path", [("rows", 32, 1, 5, 4, "resident"),
                                                      ("rows", 9, 2, 4, 7, "stream"),
                                                      ("rows", 160, 1, 8, 8, "resident"),
                                                      ("rows", 9, 3, 4, 7, "stream"),
                                                      ("planes", 7, 16, 5, 4, "stream")])
def test_small_dw_single_block(dev, layout, N, Fin, K, Fout, path):
    """Small problems (config A's N*M = 3 200 rows x 20 outputs; FinK, Fout <= 8,
    <= 16 384 rows, rows layout) form dW in ONE 256-thread block straight into
    dW (k_dw_small: no slabs, no reduction launch; profiles/r06_A): within 1e-5
    of float64 basis^T dy and deterministic across calls; the shapes past its
    limits (FinK 12, the planes layout) take the slab path, same bar."""
    from cnn_graph_amd import ops
    c = case(load_golden("golden_A.npz"))
    plan = make_plan(c, path)
    if layout == "planes" and plan.basis_elems(N, Fin, K, Fout, "planes") is None:
        pytest.skip("planes layout does not apply")
    rng = np.random.default_rng(5 + N)
    x = t(rng.random((N, c["M"], Fin), dtype=np.float32), dev)
    W = t((rng.standard_normal((Fin * K, Fout)) * 0.1).astype(np.float32), dev)
    dy = t(rng.standard_normal((N, c["M"], Fout)).astype(np.float32), dev)
    r = ops.ChebRunner(plan, N, Fin, K, Fout, dev, basis_layout=layout)
    r.forward(x, W)
    _, dW1 = r.backward(dy, W)
    dW1 = dW1.clone()
    _, dW2 = r.backward(dy, W)
    torch.cuda.synchronize()
    assert torch.equal(dW1, dW2)
    b64 = r.basis_rows().cpu().numpy().astype(np.float64)
    ref = b64.T @ dy.cpu().numpy().astype(np.float64).reshape(-1, Fout)
    assert O.normwise_err(dW1.cpu().numpy(), ref) < TOL
