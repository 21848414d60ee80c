"""Generate the golden fixtures under tests/golden/ by IMPORTING the reference.

Run in the build container only (the reference is not present on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What comes from the reference itself (imported read-only from
/root/reference/lib):
  * graph construction: lib/graph.py grid / distance_* / adjacency / laplacian
  * L~ = lib/graph.py::rescale_L(csr_matrix(L), 2)      (lib/graph_conv.py:148-149)
  * the fp32 Chebyshev basis: lib/graph.py::chebyshev  (lib/graph.py:241-258)
  * coarsening: lib/coarsening.py::metis / compute_perm / perm_data
TF-only semantics (layout transposes, MatMul, autodiff, MaxPool) cannot be run
here (tensorflow is not installed); their expected values are float64 NumPy
restatements of the reference source text (keys ``*_ref``).
"""
import os
import sys

import numpy as np
import scipy.sparse

REF = "/root/reference/lib"
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REF)
sys.dont_write_bytecode = True

import graph  # noqa: E402  (reference lib/graph.py)
import coarsening  # noqa: E402  (reference lib/coarsening.py)


def layout_in(x):
    N, M, Fin = x.shape
    return np.ascontiguousarray(np.transpose(x, (1, 2, 0)).reshape(M, Fin * N))


def layout_basis(Xt, N, M, Fin, K):
    return np.ascontiguousarray(np.transpose(Xt.reshape(K, M, Fin, N), (3, 1, 2, 0)).reshape(N * M, Fin * K))


def trunc_normal(rng, shape, std=0.1):
    w = rng.normal(0, std, size=shape)
    bad = np.abs(w) > 2 * std
    while bad.any():
        w[bad] = rng.normal(0, std, size=bad.sum())
        bad = np.abs(w) > 2 * std
    return w.astype(np.float32)


def truth_f64(Lt, basis, W, dy, N, M, Fin, K):
    """float64 truth of y, dx, dW (restated TF semantics)."""
    Fout = W.shape[1]
    y = (basis.astype(np.float64) @ W.astype(np.float64)).reshape(N, M, Fout)
    dY2 = dy.reshape(N * M, Fout).astype(np.float64)
    dW = basis.astype(np.float64).T @ dY2
    dA = dY2 @ W.astype(np.float64).T
    D = np.transpose(dA.reshape(N, M, Fin, K), (3, 1, 2, 0)).reshape(K, M, Fin * N)
    LT = scipy.sparse.csr_matrix(Lt, dtype=np.float64).T.tocsr()
    G = [None] * (K + 2)
    G[K] = G[K + 1] = np.zeros((M, Fin * N))
    for k in range(K - 1, -1, -1):
        G[k] = D[k] + (2.0 if k >= 1 else 1.0) * (LT @ G[k + 1]) - G[k + 2]
    dx = np.ascontiguousarray(np.transpose(G[0].reshape(M, Fin, N), (2, 0, 1)))
    return y, dx, dW


def cheb_case(L, N, Fin, K, Fout, seed, fake_rows=None):
    """One filter case: inputs + reference basis + float64 truth."""
    rng = np.random.default_rng(seed)
    M = L.shape[0]
    Lt = graph.rescale_L(scipy.sparse.csr_matrix(L, copy=True), lmax=2)
    assert Lt.has_sorted_indices
    x = rng.random((N, M, Fin), dtype=np.float32)
    if fake_rows is not None:
        x[:, fake_rows, :] = 0
    W = trunc_normal(rng, (Fin * K, Fout))
    dy = rng.normal(0, 1, (N, M, Fout)).astype(np.float32)
    X0 = layout_in(x)
    Xt = graph.chebyshev(Lt, X0, K)            # <- the reference's own fp32 recurrence
    basis = layout_basis(Xt, N, M, Fin, K)
    y, dx, dW = truth_f64(Lt, basis, W, dy, N, M, Fin, K)
    return dict(M=M, N=N, Fin=Fin, K=K, Fout=Fout,
                Lt_rowptr=Lt.indptr.astype(np.int32), Lt_col=Lt.indices.astype(np.int32),
                Lt_val=Lt.data.astype(np.float32),
                x=x, W=W, dy=dy, basis=basis,
                # float64 truth, stored rounded to fp32 (6e-8 rel << the 1e-5 bar)
                y_ref=y.astype(np.float32), dx_ref=dx.astype(np.float32), dW_ref=dW)


def save(name, **arrs):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrs)
    print(f"wrote {path} ({os.path.getsize(path) / 1024:.0f} KB)")


def csr_arrays(prefix, A):
    A = scipy.sparse.csr_matrix(A)
    return {f"{prefix}_indptr": A.indptr.astype(np.int32), f"{prefix}_indices": A.indices.astype(np.int32),
            f"{prefix}_data": A.data, f"{prefix}_shape": np.array(A.shape, np.int64)}


def config_a():
    """usage.ipynb cells 3/7 with k=4: M=100, K=5, Fin=1, Fout=4, N=32."""
    np.random.seed(0)
    d, n, c = 100, 10000, 5
    X = np.random.normal(0, 1, (n, d)).astype(np.float32)
    X += np.linspace(0, 1, c).repeat(d // c)
    Xtr = X[: n // 2]
    dist, idx = graph.distance_scipy_spatial(Xtr.T, k=4, metric="euclidean")
    A = graph.adjacency(dist, idx).astype(np.float32)
    L = graph.laplacian(A, normalized=True)
    case = cheb_case(L, N=32, Fin=1, K=5, Fout=4, seed=2017)
    case2 = cheb_case(L, N=8, Fin=3, K=4, Fout=5, seed=2018)   # Fin>1 layout coverage
    case3 = cheb_case(L, N=4, Fin=2, K=1, Fout=3, seed=2019)   # K=1 (basis = identity)
    case4 = cheb_case(L, N=4, Fin=1, K=2, Fout=3, seed=2020)   # K=2 (no recurrence)
    out = {**case, **{f"fin3_{k}": v for k, v in case2.items()},
           **{f"k1_{k}": v for k, v in case3.items()}, **{f"k2_{k}": v for k, v in case4.items()}}
    out.update(csr_arrays("L", L))
    save("golden_A.npz", **out)


def config_b():
    """MNIST recipe (nips2016/mnist.ipynb:89-91): grid(28) 8-NN,
    seed 10, coarsen(levels=4) -> M=976.  Also records the coarsening run."""
    np.random.seed(10)
    z = graph.grid(28)
    dist, idx = graph.distance_sklearn_metrics(z, k=8, metric="euclidean")
    A = graph.adjacency(dist, idx)
    A = graph.replace_random_edges(A, 0)
    # coarsening.coarsen(A, 4) = metis + compute_perm + perm_adjacency; run the
    # pieces to capture the level-0 visit order (unseeded permutation :56) and
    # the tie-sensitive argsort orders of later levels (:112-113).
    rid0 = np.random.permutation(range(A.shape[0]))
    graphs, parents = coarsening.metis(A, 4, rid=rid0)
    rids = [rid0] + [np.argsort(np.array(g.sum(axis=0)).squeeze()) for g in graphs[1:-1]]
    perms = coarsening.compute_perm(parents)
    G0 = graphs[0].tocoo()
    G0.setdiag(0)
    G0 = coarsening.perm_adjacency(G0, perms[0]).tocsr()
    G0.eliminate_zeros()
    L = graph.laplacian(G0, normalized=True)
    M = L.shape[0]
    assert M == 976, M
    fake = np.nonzero(np.asarray(perms[0]) >= A.shape[0])[0]
    case = cheb_case(L, N=8, Fin=1, K=25, Fout=32, seed=2017, fake_rows=fake)
    # perm_data on real MNIST-shaped data (N=4 x 784) through the reference
    data = np.random.default_rng(7).random((4, A.shape[0]), dtype=np.float32)
    pdata = coarsening.perm_data(data, perms[0])
    out = dict(case)
    out.update(csr_arrays("A", A))
    out.update(csr_arrays("L", L))
    out["perm0"] = np.asarray(perms[0], np.int32)
    for i, p in enumerate(parents):
        out[f"parents{i}"] = np.asarray(p, np.int32)
    for i, r in enumerate(rids):
        out[f"rid{i}"] = np.asarray(r, np.int64)
    for i, p in enumerate(perms):
        out[f"perm_level{i}"] = np.asarray(p, np.int32)
    out["fake_rows"] = fake.astype(np.int32)
    out["pdata_in"] = data
    out["pdata_out"] = pdata
    save("golden_B.npz", **out)


def config_e():
    """gconv-LSTM graph: grid(32) 8-NN (nips2016/gconvTest.py:62-79), Fin=2, K=3."""
    z = graph.grid(32)
    dist, idx = graph.distance_sklearn_metrics(z, k=8, metric="euclidean")
    A = graph.adjacency(dist, idx)
    L = graph.laplacian(A, normalized=True)
    case = cheb_case(L, N=4, Fin=2, K=3, Fout=32, seed=2021)
    save("golden_E.npz", **case)


def config_c():
    """20NEWS-like vocabulary graph: 10 000 x 100 Gaussian
    embeddings (np.random.seed(0)), cosine 16-NN via the reference's
    distance_sklearn_metrics / adjacency / laplacian -> nnz(L~) = 182 466,
    max row nnz 32.  Streaming-path sizes (M > 2048)."""
    np.random.seed(0)
    X = np.random.normal(0, 1, (10000, 100)).astype(np.float32)
    dist, idx = graph.distance_sklearn_metrics(X, k=16, metric="cosine")
    A = graph.adjacency(dist, idx)
    L = graph.laplacian(A, normalized=True)
    case = cheb_case(L, N=2, Fin=1, K=5, Fout=8, seed=2022)      # layer 1 (Fin=1)
    case2 = cheb_case(L, N=1, Fin=3, K=5, Fout=4, seed=2023)     # Fin>1 layout
    assert int(case["Lt_rowptr"][-1]) == 182466
    out = {**case, **{f"fin3_{k}": v for k, v in case2.items()
                      if not k.startswith("Lt_")}}
    save("golden_C.npz", **out)


def misc():
    # (iii) compute_perm known answer, lib/coarsening.py:216-217
    parents = [np.array([4, 1, 1, 2, 2, 3, 0, 0, 3]), np.array([2, 1, 0, 1, 0])]
    kp = coarsening.compute_perm(parents)
    # (iv) max-pool with ties (TF first-max rule restated; TF boundary unpinned)
    rng = np.random.default_rng(5)
    xp = rng.integers(0, 3, size=(3, 16, 5)).astype(np.float32)   # many ties
    xp[:, 4:8, :] = 0.0                                            # all-tie windows
    # (v) spectral equivalence, trials/1_learning_filters.ipynb:1045-1163 (fp64, M=100 grid 4-NN)
    z = graph.grid(10, dtype=np.float64)
    dist, idx = graph.distance_scipy_spatial(z, k=4)
    A = graph.adjacency(dist, idx)
    L = graph.laplacian(A, normalized=True)
    Xs = np.random.default_rng(11).normal(0, 1, (100, 6))
    Lt = graph.rescale_L(scipy.sparse.csr_matrix(L, copy=True), lmax=2)
    Xt = graph.chebyshev(Lt, Xs, 6)       # fp64 basis from the reference
    save("golden_misc.npz",
         kp0=np.array(kp[0], np.int32), kp1=np.array(kp[1], np.int32), kp2=np.array(kp[2], np.int32),
         kp_parents0=parents[0].astype(np.int32), kp_parents1=parents[1].astype(np.int32),
         pool_x=xp, spec_X=Xs, spec_basis=Xt, **csr_arrays("spec_L", L))


if __name__ == "__main__":
    # optional argv: the fixtures to (re)generate, e.g. `make_golden.py config_c`
    todo = sys.argv[1:] or ["config_a", "config_b", "config_e", "config_c", "misc"]
    for name in todo:
        globals()[name]()
