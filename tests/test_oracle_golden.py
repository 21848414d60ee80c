"""Pin the CPU oracle to the reference's own outputs (golden fixtures made by
importing /root/reference/lib in the build container, tests/golden/make_golden.py)."""
import numpy as np
import pytest
import scipy.sparse
import torch

from oracle import cheb_oracle as O
from conftest import CASES, CASE_IDS, case, load_golden

TOL = 1e-5  # max-abs-normalised, the north-star filter-output bar


def csr_from(g, prefix):
    return scipy.sparse.csr_matrix((g[f"{prefix}_data"], g[f"{prefix}_indices"], g[f"{prefix}_indptr"]),
                                   shape=tuple(g[f"{prefix}_shape"]))


@pytest.mark.parametrize("fname,prefix", CASES, ids=CASE_IDS)
def test_basis_bit_exact_vs_reference_chebyshev(fname, prefix):
    """oracle basis == lib/graph.py::chebyshev (+ layout of lib/graph_conv.py:170-172), bit for bit."""
    c = case(load_golden(fname), prefix)
    basis, _ = O.cheb_forward(c["x"], c["Lt_rowptr"], c["Lt_col"], c["Lt_val"], c["W"], c["K"])
    assert basis.dtype == np.float32
    assert np.array_equal(basis, c["basis"])


@pytest.mark.parametrize("fname", ["golden_A.npz", "golden_B.npz"])
def test_rescale_bit_exact(fname):
    """oracle.rescale_L + canonical order == the reference's L~ (lib/graph.py:232-238)."""
    g = load_golden(fname)
    L = csr_from(g, "L")
    rp, ci, v = O.canonical_csr(O.rescale_L(L, 2))
    assert np.array_equal(rp, g["Lt_rowptr"]) and np.array_equal(ci, g["Lt_col"])
    assert np.array_equal(v, g["Lt_val"])


def test_rescale_lmax_not_2_scales_by_fp32_reciprocal():
    g = load_golden("golden_A.npz")
    L = csr_from(g, "L")
    Lt = O.rescale_L(L, 3.0)
    ref = (L.astype(np.float32) * np.float32(1.0 / 1.5)) - scipy.sparse.identity(L.shape[0], dtype=np.float32)
    assert np.array_equal(Lt.toarray(), ref.toarray())
    assert L.data.dtype == np.float32  # caller's L untouched
    assert np.array_equal(csr_from(g, "L").data, L.data)


@pytest.mark.parametrize("fname,prefix", CASES, ids=CASE_IDS)
def test_forward_backward_vs_f64_truth(fname, prefix):
    c = case(load_golden(fname), prefix)
    basis, y = O.cheb_forward(c["x"], c["Lt_rowptr"], c["Lt_col"], c["Lt_val"], c["W"], c["K"])
    assert O.normwise_err(y, c["y_ref"]) < 1e-6
    dx, dW = O.cheb_backward(c["dy"], basis, c["W"], c["Lt_rowptr"], c["Lt_col"], c["Lt_val"],
                             c["N"], c["M"], c["Fin"], c["K"])
    assert O.normwise_err(dx, c["dx_ref"]) < 1e-6
    assert O.normwise_err(dW, c["dW_ref"]) < 1e-10


@pytest.mark.parametrize("prefix", ["", "fin3_", "k2_"])
def test_backward_matches_independent_autograd(prefix):
    """The analytic Clenshaw backward equals torch autograd of a dense fp64
    restatement of chebyshev5 (transposes + recurrence + matmul)."""
    c = case(load_golden("golden_A.npz"), prefix)
    N, M, Fin, K, Fout = c["N"], c["M"], c["Fin"], c["K"], c["Fout"]
    Ld = torch.tensor(scipy.sparse.csr_matrix((c["Lt_val"], c["Lt_col"], c["Lt_rowptr"]), shape=(M, M))
                      .toarray(), dtype=torch.float64)
    x = torch.tensor(c["x"], dtype=torch.float64, requires_grad=True)
    W = torch.tensor(c["W"], dtype=torch.float64, requires_grad=True)
    x0 = x.permute(1, 2, 0).reshape(M, Fin * N)
    Ts = [x0]
    if K > 1:
        Ts.append(Ld @ x0)
    for k in range(2, K):
        Ts.append(2 * (Ld @ Ts[-1]) - Ts[-2])
    B = torch.stack(Ts).reshape(K, M, Fin, N).permute(3, 1, 2, 0).reshape(N * M, Fin * K)
    y = (B @ W).reshape(N, M, Fout)
    y.backward(torch.tensor(c["dy"], dtype=torch.float64))
    basis, _ = O.cheb_forward(c["x"], c["Lt_rowptr"], c["Lt_col"], c["Lt_val"], c["W"], K)
    dx, dW = O.cheb_backward(c["dy"], basis, c["W"], c["Lt_rowptr"], c["Lt_col"], c["Lt_val"], N, M, Fin, K)
    assert O.normwise_err(dx, x.grad.numpy()) < 1e-6
    assert O.normwise_err(dW, W.grad.numpy()) < 1e-6


def test_spmm_order_matches_scipy_dot():
    """The slot-wise SpMM reproduces scipy csr_matvecs (used by L.dot) bitwise."""
    g = load_golden("golden_B.npz")
    M = int(g["M"])
    A = scipy.sparse.csr_matrix((g["Lt_val"], g["Lt_col"], g["Lt_rowptr"]), shape=(M, M))
    X = np.random.default_rng(3).standard_normal((M, 37)).astype(np.float32)
    assert np.array_equal(O.spmm_seq(g["Lt_rowptr"], g["Lt_col"], g["Lt_val"], X), A.dot(X))


def test_k1_basis_is_identity_layout():
    """trials/1_learning_filters.ipynb:1067 -- the K=1 basis is the input itself."""
    c = case(load_golden("golden_A.npz"), "k1_")
    N, M, Fin = c["N"], c["M"], c["Fin"]
    assert np.array_equal(c["basis"].reshape(N, M, Fin), c["x"])


def test_spectral_equivalence_fp64():
    """trials/1_learning_filters.ipynb:1115-1163: basis filter == full spectral
    filter U g(L~) U^T x at 1e-10 for unit and random coefficient vectors."""
    g = load_golden("golden_misc.npz")
    L = csr_from(g, "spec_L")
    X = g["spec_X"]
    Xt_ref = g["spec_basis"]                   # reference lib/graph.py::chebyshev, fp64
    rp, ci, v = O.canonical_csr(O.rescale_L(L, 2))
    Xt = O.chebyshev_basis(rp, ci, v.astype(np.float64), X, 6)
    Lt64 = O.rescale_L(L, 2)
    Xt64 = O.chebyshev_basis(Lt64.indptr, Lt64.indices, Lt64.data, X, 6)
    assert np.array_equal(Xt64, Xt_ref)
    rng = np.random.default_rng(0)
    for coeffs in ([1.0], [1, 0, 0, 0], [0, 0, 0, 1], list(rng.uniform(0, 5, 6))):
        K = len(coeffs)
        y_basis = np.tensordot(np.asarray(coeffs), Xt_ref[:K], axes=1)
        y_full = O.chebyshev_spectral(L, X, coeffs)
        np.testing.assert_allclose(y_basis, y_full, atol=1e-10)
    assert Xt.shape == Xt_ref.shape


def test_compute_perm_known_answer():
    """lib/coarsening.py:216-217."""
    g = load_golden("golden_misc.npz")
    got = O.compute_perm([g["kp_parents0"], g["kp_parents1"]])
    assert got == [list(g["kp0"]), list(g["kp1"]), list(g["kp2"])]
    assert got == [[3, 4, 0, 9, 1, 2, 5, 8, 6, 7, 10, 11], [2, 4, 1, 3, 0, 5], [0, 1, 2]]


def test_metis_with_recorded_visit_orders_matches_reference():
    g = load_golden("golden_B.npz")
    A = csr_from(g, "A")
    rids = [g[f"rid{i}"] for i in range(4)]
    graphs, parents = O.metis(A, 4, rids)
    for i, p in enumerate(parents):
        assert np.array_equal(p, g[f"parents{i}"])
    perms = O.compute_perm(parents)
    assert np.array_equal(np.asarray(perms[0]), g["perm0"])
    assert [len(p) for p in perms] == [976, 488, 244, 122, 61]


def test_perm_data_vs_reference():
    g = load_golden("golden_B.npz")
    out = O.perm_data(g["pdata_in"], g["perm0"])
    assert np.array_equal(out, g["pdata_out"].astype(np.float32))


def test_maxpool_first_max_rule():
    g = load_golden("golden_misc.npz")
    x = g["pool_x"]
    for p in (2, 4, 8):
        y, arg = O.mpool1_forward(x, p)
        N, M, F = x.shape
        xw = x.reshape(N, M // p, p, F)
        assert np.array_equal(y, xw.max(axis=2))
        # argmax is the FIRST index of the maximum inside each window
        first = np.argmax(xw == xw.max(axis=2, keepdims=True), axis=2)
        assert np.array_equal(arg, first + (np.arange(M // p) * p)[None, :, None])
        dy = np.random.default_rng(p).standard_normal(y.shape).astype(np.float32)
        dx = O.mpool1_backward(dy, arg, M)
        assert np.isclose(dx.sum(), dy.sum(), atol=1e-4)
        assert (dx != 0).sum() <= dy.size


@pytest.mark.parametrize("prefix", ["", "fin3_"])
def test_config_c_oracle_vs_reference(prefix):
    """Config C (10 000-vertex cosine 16-NN graph built by the reference's
    lib/graph.py): oracle basis bit-equal to lib/graph.py::chebyshev, outputs
    vs the float64 truth."""
    g = load_golden("golden_C.npz")
    c = case(g, prefix)
    rp, ci, v = g["Lt_rowptr"], g["Lt_col"], g["Lt_val"]
    basis, y = O.cheb_forward(c["x"], rp, ci, v, c["W"], c["K"])
    assert np.array_equal(basis, c["basis"])
    assert O.normwise_err(y, c["y_ref"]) < 1e-6
    dx, dW = O.cheb_backward(c["dy"], basis, c["W"], rp, ci, v, c["N"], int(g["M"]), c["Fin"], c["K"])
    assert O.normwise_err(dx, c["dx_ref"]) < 1e-6
    assert O.normwise_err(dW, c["dW_ref"]) < 1e-10
