"""Product coarsening (cnn_graph_amd.coarsening: native Graclus matching and
tree order in libcheb_mi355.so) against the reference's recorded run
(tests/golden/golden_B.npz, made by importing /root/reference/lib/coarsening.py)
and the oracle restatement.  Host-only: runs without a GPU."""
import numpy as np
import pytest
import scipy.sparse

from oracle import cheb_oracle as O
from conftest import load_golden

pytestmark = pytest.mark.usefixtures("built_lib")


def _csr(g, prefix):
    return scipy.sparse.csr_matrix((g[f"{prefix}_data"], g[f"{prefix}_indices"], g[f"{prefix}_indptr"]),
                                   shape=tuple(g[f"{prefix}_shape"]))


def test_compute_perm_known_answer():
    """The reference's own assertion, lib/coarsening.py:216-217."""
    from cnn_graph_amd import coarsening as C
    got = C.compute_perm([np.array([4, 1, 1, 2, 2, 3, 0, 0, 3]), np.array([2, 1, 0, 1, 0])])
    assert got == [[3, 4, 0, 9, 1, 2, 5, 8, 6, 7, 10, 11], [2, 4, 1, 3, 0, 5], [0, 1, 2]]
    g = load_golden("golden_misc.npz")
    assert got == [list(g["kp0"]), list(g["kp1"]), list(g["kp2"])]


def test_metis_matches_recorded_reference_run():
    from cnn_graph_amd import coarsening as C
    g = load_golden("golden_B.npz")
    A = _csr(g, "A")
    rids = [g[f"rid{i}"] for i in range(4)]
    graphs, parents = C.metis(A, 4, rids=rids)
    for i, p in enumerate(parents):
        assert np.array_equal(p, g[f"parents{i}"]), f"level {i}"
    perms = C.compute_perm(parents)
    for i, p in enumerate(perms):
        assert np.array_equal(np.asarray(p), g[f"perm_level{i}"]), f"perm level {i}"
    assert [len(p) for p in perms] == [976, 488, 244, 122, 61]


def test_metis_level0_rid_only_reproduces_argsort_levels():
    """Only the level-0 permutation injected: later levels take the reference's
    own np.argsort of the degrees, as recorded."""
    from cnn_graph_amd import coarsening as C
    g = load_golden("golden_B.npz")
    _, parents = C.metis(_csr(g, "A"), 4, rid=g["rid0"])
    for i, p in enumerate(parents):
        assert np.array_equal(p, g[f"parents{i}"]), f"level {i}"


def test_coarsen_graph_gives_reference_laplacian():
    """coarsen -> level-0 graph -> laplacian == the golden L of config B (bitwise)."""
    from cnn_graph_amd import coarsening as C, graph
    g = load_golden("golden_B.npz")
    rids = [g[f"rid{i}"] for i in range(4)]
    graphs, perm = C.coarsen(_csr(g, "A"), 4, rids=rids, verbose=False)
    assert np.array_equal(np.asarray(perm), g["perm0"])
    assert [G.shape[0] for G in graphs] == [976, 488, 244, 122, 61]
    L = graph.laplacian(graphs[0], normalized=True)
    Lg = _csr(g, "L")
    L.sort_indices()
    Lg.sort_indices()
    assert np.array_equal(L.indptr, Lg.indptr) and np.array_equal(L.indices, Lg.indices)
    assert np.array_equal(L.data.view(np.uint32), Lg.data.view(np.uint32))


def test_perm_data_host_matches_reference():
    from cnn_graph_amd import coarsening as C
    g = load_golden("golden_B.npz")
    out = C.perm_data(g["pdata_in"], g["perm0"])
    assert out.dtype == np.float64  # the reference's np.empty
    assert np.array_equal(out, g["pdata_out"])


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_graclus_matches_oracle_on_random_graphs(dtype, seed):
    """Random symmetric graphs with quantised weights (many score ties), vs the
    oracle's pure-loop restatement of lib/coarsening.py:119-165."""
    from cnn_graph_amd import coarsening as C
    rng = np.random.default_rng(seed)
    M = 300
    A = scipy.sparse.random(M, M, density=0.02, random_state=seed, dtype=np.float64)
    A.data = np.round(A.data * 4) / 4 + 0.25
    A = scipy.sparse.csr_matrix(A + A.T).astype(dtype)
    A.setdiag(0)
    A.eliminate_zeros()
    # keep the last row non-empty (the reference infers N from it)
    A = A + scipy.sparse.csr_matrix(([dtype(1), dtype(1)], ([M - 1, 0], [0, M - 1])), shape=(M, M))
    A = scipy.sparse.csr_matrix(A, dtype=dtype)
    degree = np.array(A.sum(axis=0) - A.diagonal()).squeeze()
    r, c, v = scipy.sparse.find(A)
    p = np.argsort(r)
    rr, cc, vv = r[p], c[p], v[p]
    rid = rng.permutation(M)
    got = C.metis_one_level(rr, cc, vv, rid, degree)
    want = O.metis_one_level(rr, cc, vv, rid, degree)
    assert np.array_equal(got, want)


def test_graclus_bad_visit_order_raises():
    from cnn_graph_amd import coarsening as C
    from cnn_graph_amd._lib import CGError
    rr = np.array([0, 0, 1, 2], np.int32)
    cc = np.array([1, 2, 0, 0], np.int32)
    vv = np.ones(4, np.float32)
    with pytest.raises(CGError, match="out of range"):
        C.metis_one_level(rr, cc, vv, np.array([0, 7, 1]), np.ones(3, np.float32))


def test_compute_perm_rejects_three_children():
    from cnn_graph_amd import coarsening as C
    from cnn_graph_amd._lib import CGError
    with pytest.raises(CGError, match="> 2 children"):
        C.compute_perm([np.array([0, 0, 0, 1])])
