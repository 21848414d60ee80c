"""Channel-group resident backward with dBasis formed in the kernel
(cheb_group.hip::k_grp_clen_dy: the whole reverse recurrence of one sample x 8
channels in LDS, D_k = dy W_k^T on MFMA per group of four orders, no dBasis
planes).  Bars: dx BITWISE equal to the one-launch-per-step streaming path
(plan variant 'steps': k_rowgemm dBasis planes + k_clenshaw_step, the same
MFMA operation sequence and the same recurrence expressions), dx and dW within
1e-5 of the float64 oracle (oracle/cheb_oracle.py::cheb_backward, restating
TF autodiff of lib/graph_conv.py:164-176), dx accumulation (the residual
block's dx +=) exact."""
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


def _t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(dev)


# (golden graph, N, Fin, K, Fout): config R's hidden layer (M = 1024, K = 20),
# a partial order group (K = 7, 2), Fout = 64 (two 16-step chunks per half),
# a graph whose last row tile is ragged (config B, M = 976), Fout = 2 (the
# ResGNN output layer: one MFMA step per tile)
CASES = [("golden_E.npz", 3, 32, 20, 32), ("golden_E.npz", 2, 16, 7, 64),
         ("golden_E.npz", 4, 8, 2, 32), ("golden_B.npz", 3, 24, 5, 32),
         ("golden_B.npz", 2, 32, 20, 32), ("golden_B.npz", 2, 8, 1, 32),
         ("golden_E.npz", 3, 32, 20, 2), ("golden_B.npz", 2, 16, 5, 2)]


@pytest.mark.parametrize("gname,N,Fin,K,Fout", CASES)
def test_group_clenshaw_fused_dbasis(dev, cg_opts, gname, N, Fin, K, Fout):
    """The fused-dBasis group Clenshaw (auto) against the steps path: dx
    bitwise equal when the steps path's dBasis GEMM is the f32-MFMA k_rowgemm
    (CG_OPT_GEMM_X3 = 0: same products, same order); with the default
    split-bf16 row GEMM the steps path's dx / dW within 1e-5 of float64."""
    from cnn_graph_amd import ops
    from cnn_graph_amd.plan import ChebPlan
    c = case(load_golden(gname))
    M = c["M"]
    Lt = scipy.sparse.csr_matrix((c["Lt_val"], c["Lt_col"], c["Lt_rowptr"]), shape=(M, M))
    rng = np.random.default_rng(N * 100 + Fin * 10 + K)
    x = rng.standard_normal((N, M, Fin)).astype(np.float32)
    W = (rng.standard_normal((Fin * K, Fout)) * 0.1).astype(np.float32)
    dy = rng.standard_normal((N, M, Fout)).astype(np.float32)
    xt, Wt, dyt = _t(x, dev), _t(W, dev), _t(dy, dev)
    out = {}
    for variant, x3 in (("auto", 0), ("steps", 0), ("steps_x3", 1)):
        cg_opts("gemm_x3", x3)
        plan = ChebPlan(Lt, device=0, path="stream", variant=variant.split("_")[0])
        r = ops.ChebRunner(plan, N, Fin, K, Fout, dev, basis_layout="rows")
        r.forward(xt, Wt)
        r.backward(dyt, Wt)
        torch.cuda.synchronize()
        out[variant] = (r.basis.clone(), r.dx.clone(), r.dW.clone())
    assert torch.equal(out["auto"][0], out["steps"][0])
    assert torch.equal(out["auto"][1], out["steps"][1]), "dx differs from the steps path"
    basis = out["auto"][0].cpu().numpy()
    odx, odW = O.cheb_backward(dy, basis, W, c["Lt_rowptr"], c["Lt_col"], c["Lt_val"], N, M, Fin, K)
    for v in ("auto", "steps_x3"):
        assert O.normwise_err(out[v][1].cpu().numpy(), odx) < TOL
        assert O.normwise_err(out[v][2].cpu().numpy(), odW) < TOL


def test_group_clenshaw_fused_dx_accumulate(dev):
    """cg_cheb_backward_ex's dx += (the residual block): dx0 + G_0 exactly."""
    from cnn_graph_amd import _lib, ops
    from cnn_graph_amd.plan import ChebPlan
    c = case(load_golden("golden_E.npz"))
    M = c["M"]
    Lt = scipy.sparse.csr_matrix((c["Lt_val"], c["Lt_col"], c["Lt_rowptr"]), shape=(M, M))
    N, Fin, K, Fout = 2, 32, 6, 32
    rng = np.random.default_rng(5)
    x = _t(rng.standard_normal((N, M, Fin)), dev)
    W = _t(rng.standard_normal((Fin * K, Fout)) * 0.1, dev)
    dy = _t(rng.standard_normal((N, M, Fout)), dev)
    dx0 = _t(rng.standard_normal((N, M, Fin)), dev)
    plan = ChebPlan(Lt, device=0, path="stream")
    r = ops.ChebRunner(plan, N, Fin, K, Fout, dev, basis_layout="rows")
    r.forward(x, W)
    r.backward(dy, W)
    torch.cuda.synchronize()
    ref = dx0 + r.dx
    dxa = dx0.clone()
    dW = torch.empty_like(W)
    _lib.check("cg_cheb_backward_ex", _lib.lib().cg_cheb_backward_ex(
        plan.handle, N, Fin, K, Fout, dy.data_ptr(), None, _lib.CG_ACT_NONE,
        r.basis.data_ptr(), W.data_ptr(), dxa.data_ptr(), 1, dW.data_ptr(), None,
        r.bws.data_ptr(), r.bwd_bytes, torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    assert torch.equal(dxa, ref)
    assert torch.equal(dW, r.dW)


@pytest.mark.parametrize("gname,N,Fin,K,Fout", [("golden_E.npz", 3, 32, 20, 24), ("golden_B.npz", 2, 16, 5, 40)])
def test_group_clenshaw_packed_columns_bitwise(dev, cg_opts, gname, N, Fin, K, Fout):
    """k_grp_clen (the dBasis-planes variant, Fout outside the fused kernel's
    2 / 32 / 64) with the rows' columns packed in registers: dx bitwise equal to
    the steps path.  (Its LDS-columns alternative, CG_OPT_GRP_PC = 0, exists in
    the ablation build only since round 6; the release library rejects it.)"""
    from cnn_graph_amd import ops
    from cnn_graph_amd.plan import ChebPlan
    c = case(load_golden(gname))
    M = c["M"]
    Lt = scipy.sparse.csr_matrix((c["Lt_val"], c["Lt_col"], c["Lt_rowptr"]), shape=(M, M))
    rng = np.random.default_rng(N + Fin + K + Fout)
    xt = _t(rng.standard_normal((N, M, Fin)), dev)
    Wt = _t(rng.standard_normal((Fin * K, Fout)) * 0.1, dev)
    dyt = _t(rng.standard_normal((N, M, Fout)), dev)
    out = {}
    for name, variant in (("pc", "auto"), ("steps", "steps")):
        plan = ChebPlan(Lt, device=0, path="stream", variant=variant)
        r = ops.ChebRunner(plan, N, Fin, K, Fout, dev, basis_layout="rows")
        r.forward(xt, Wt)
        r.backward(dyt, Wt)
        torch.cuda.synchronize()
        out[name] = r.dx.clone()
    assert torch.equal(out["pc"], out["steps"])
    from cnn_graph_amd import _lib
    with pytest.raises(_lib.CGError):
        cg_opts("grp_pc", "0")


@pytest.mark.parametrize("gname,N,Fin,K,Fout", [("golden_E.npz", 3, 32, 20, 32), ("golden_B.npz", 2, 16, 5, 32),
                                                ("golden_B.npz", 2, 32, 7, 20)])
def test_group_fwd_paired_metadata_bitwise(dev, cg_opts, gname, N, Fin, K, Fout):
    """k_grp16_fwd with the CSR metadata read two entries per LDS access
    (lds_row_spmm_w; rows start at both parities of the CSR) against the steps
    path: basis planes bitwise equal, y within 1e-6 (another contraction order).
    (The one-entry-per-access alternative, CG_OPT_SPMM_PW = 0, exists in the
    ablation build only since round 6.)"""
    from cnn_graph_amd import ops
    from cnn_graph_amd.plan import ChebPlan
    c = case(load_golden(gname))
    M = c["M"]
    Lt = scipy.sparse.csr_matrix((c["Lt_val"], c["Lt_col"], c["Lt_rowptr"]), shape=(M, M))
    assert (np.asarray(c["Lt_rowptr"][:-1]) % 2 == 1).any()
    rng = np.random.default_rng(N + Fin + K + Fout + 11)
    cg_opts("gemm_x3", 0)  # the steps path's y on the f32-MFMA row GEMM
    xt = _t(rng.standard_normal((N, M, Fin)), dev)
    Wt = _t(rng.standard_normal((Fin * K, Fout)) * 0.1, dev)
    out = {}
    for name, variant in (("grp", "auto"), ("steps", "steps")):
        plan = ChebPlan(Lt, device=0, path="stream", variant=variant)
        r = ops.ChebRunner(plan, N, Fin, K, Fout, dev, basis_layout="planes")
        r.forward(xt, Wt)
        torch.cuda.synchronize()
        out[name] = (r.basis.clone(), r.y.clone())
    assert torch.equal(out["grp"][0], out["steps"][0])
    err = O.normwise_err(out["grp"][1].cpu().numpy(), out["steps"][1].cpu().numpy().astype(np.float64))
    assert err < 1e-6, err
    from cnn_graph_amd import _lib
    with pytest.raises(_lib.CGError):
        cg_opts("spmm_pw", "0")
