"""The functional filter ``cheby_conv(x, L, lmax, feat_out, K, W)``
(lib/filter.py:45-95, duplicated at lib/models.py:416-460 and
lib/gconvRNN.py:27-71) through torch autograd on the HIP path, for lmax = 2
(what graph.lmax returns for normalized Laplacians) and lmax = 3 (the rescale
L~ = L / 1.5 - I of lib/graph.py:232-238 with a non-trivial scale), checked
against the oracle built from the SAME rescaled Laplacian: basis bit-exact
through the forward, y / dx / dW within 1e-5 normwise of float64.

Deliberate difference, documented: the reference's rescale_L divides the
caller's ``L.data`` in place (``L /= lmax / 2``), so calling cheby_conv twice
with one L and lmax != 2 rescales it twice.  Here the rescale works on a
private copy (cnn_graph_amd.graph.rescale_L) -- the first call is identical,
repeated calls do not drift -- and the caller's L is left untouched."""
import numpy as np
import pytest
import scipy.sparse

from conftest import load_golden
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


def laplacian_of(name):
    g = load_golden(name)
    return scipy.sparse.csr_matrix((g["L_data"], g["L_indices"], g["L_indptr"]),
                                   shape=tuple(g["L_shape"]))


@pytest.mark.parametrize("name,N,Fin,K,Fout", [("golden_A.npz", 32, 1, 5, 4),
                                                ("golden_A.npz", 4, 3, 4, 6),
                                                ("golden_B.npz", 16, 1, 25, 32)])
@pytest.mark.parametrize("lmax", [2.0, 3.0])
def test_cheby_conv_functional_vs_oracle(dev, name, N, Fin, K, Fout, lmax):
    from cnn_graph_amd import filter as F
    from cnn_graph_amd import ops
    from cnn_graph_amd.plan import clear_plan_cache
    L = laplacian_of(name)
    L_before = L.data.copy()
    M = L.shape[0]
    rng = np.random.default_rng(int(lmax * 10) + Fin)
    x = rng.random((N, M, Fin), dtype=np.float32)
    W = (rng.standard_normal((K * Fin, Fout)) * 0.1).astype(np.float32)
    dy = rng.standard_normal((N, M, Fout)).astype(np.float32)

    xt = torch.from_numpy(x).to(dev).requires_grad_(True)
    Wt = torch.from_numpy(W).to(dev).requires_grad_(True)
    y = F.cheby_conv(xt, L, lmax, Fout, K, Wt)
    y.backward(torch.from_numpy(dy).to(dev))
    torch.cuda.synchronize()

    rp, ci, v = O.canonical_csr(O.rescale_L(L, lmax))
    ob, oy = O.cheb_forward(x, rp, ci, v, W, K)
    odx, odW = O.cheb_backward(dy, ob, W, rp, ci, v, N, M, Fin, K)
    assert O.normwise_err(y.detach().cpu().numpy(), oy) < TOL
    assert O.normwise_err(xt.grad.cpu().numpy(), odx) < TOL
    assert O.normwise_err(Wt.grad.cpu().numpy(), odW) < TOL
    # the basis the filter ran on is the reference's fp32 recurrence over
    # rescale_L(L, lmax), bit for bit (same cached plan as cheby_conv used)
    from cnn_graph_amd.plan import plan_for
    basis, _ = ops.cheb_forward(plan_for(L, lmax=lmax, device=0), xt.detach(), None, K)
    assert np.array_equal(basis.cpu().numpy(), ob)
    assert np.array_equal(L.data, L_before), "caller's Laplacian was modified"
    clear_plan_cache()


def test_cheby_conv_creates_weight_when_none(dev):
    """W=None creates [K*feat_in, feat_out] ~ truncated_normal(0, 0.1)
    (lib/filter.py:63-64) and returns it through cheby_conv.last_weight."""
    from cnn_graph_amd import filter as F
    L = laplacian_of("golden_A.npz")
    x = torch.rand((8, L.shape[0], 2), device=dev)
    y = F.cheby_conv(x, L, 2, 5, 3, None)
    W = F.cheby_conv.last_weight
    assert tuple(W.shape) == (3 * 2, 5) and tuple(y.shape) == (8, L.shape[0], 5)
    assert float(W.detach().abs().max()) <= 0.2
