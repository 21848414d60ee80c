"""Host graph math on the path: the Laplacian and its Chebyshev rescaling.

Mirrors the reference's ``lib/graph.py`` API for the functions the Chebyshev
filter needs (callers of the reference keep calling ``graph.laplacian`` /
``graph.rescale_L``), plus the graph builders used by its drivers.  Runs once
per graph on the host (scipy), like the reference; the device only ever sees
the canonical CSR of L~ (see plan.py).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse
import scipy.spatial.distance


def grid(m, dtype=np.float32):
    """Vertex coordinates of an m x m grid graph (lib/graph.py:10-19)."""
    M = m * m
    x = np.linspace(0, 1, m, dtype=dtype)
    xx, yy = np.meshgrid(x, x)
    z = np.empty((M, 2), dtype)
    z[:, 0] = xx.reshape(M)
    z[:, 1] = yy.reshape(M)
    return z


def distance_scipy_spatial(z, k=4, metric="euclidean"):
    """Exact k-NN distances and indices (lib/graph.py:22-30)."""
    d = scipy.spatial.distance.squareform(scipy.spatial.distance.pdist(z, metric))
    idx = np.argsort(d)[:, 1:k + 1]
    d.sort()
    return d[:, 1:k + 1], idx


def distance_sklearn_metrics(z, k=4, metric="euclidean"):
    """lib/graph.py:33-41 (sklearn pairwise distances; same result as scipy)."""
    import sklearn.metrics
    d = sklearn.metrics.pairwise.pairwise_distances(z, metric=metric, n_jobs=1)
    idx = np.argsort(d)[:, 1:k + 1]
    d.sort()
    return d[:, 1:k + 1], idx


def adjacency(dist, idx):
    """Symmetric Gaussian-kernel k-NN adjacency (lib/graph.py:57-83)."""
    M, k = dist.shape
    assert dist.min() >= 0
    sigma2 = np.mean(dist[:, -1]) ** 2
    w = np.exp(-dist ** 2 / sigma2)
    W = scipy.sparse.coo_matrix((w.reshape(M * k), (np.arange(M).repeat(k), idx.reshape(M * k))),
                                shape=(M, M))
    W.setdiag(0)
    bigger = W.T > W
    W = W - W.multiply(bigger) + W.T.multiply(bigger)
    return scipy.sparse.csr_matrix(W)


def laplacian(W, normalized=True):
    """Combinatorial or normalized Laplacian (lib/graph.py:117-136).

    normalized: ``I - D^-1/2 W D^-1/2`` with ``d += spacing(0)`` so isolated
    (fake) vertices give a zero row after rescaling.  Same float operations as
    the reference (dtype of W is kept).
    """
    d = W.sum(axis=0)
    if not normalized:
        D = scipy.sparse.diags(np.asarray(d).squeeze(), 0)
        return scipy.sparse.csr_matrix(D - W)
    d = d + np.spacing(np.array(0, W.dtype))
    d = 1 / np.sqrt(d)
    D = scipy.sparse.diags(np.asarray(d).squeeze(), 0)
    I = scipy.sparse.identity(d.size, dtype=W.dtype)
    return scipy.sparse.csr_matrix(I - D * W * D)


def lmax(L, normalized=True):
    """Upper bound of the spectrum (lib/graph.py:139-145)."""
    if normalized:
        return 2
    import scipy.sparse.linalg
    return scipy.sparse.linalg.eigsh(L, k=1, which="LM", return_eigenvectors=False)[0]


def fourier(L, algo="eigh", k=1):
    """Fourier basis = EVD of the Laplacian (lib/graph.py:148-166): (lamb, U)
    with eigenvalues ascending and U[:, i] the i-th eigenvector.  Same NumPy /
    SciPy routines as the reference, so U is the reference's U."""
    def sort(lamb, U):
        idx = lamb.argsort()
        return lamb[idx], U[:, idx]

    if algo == "eig":
        lamb, U = np.linalg.eig(L.toarray())
        lamb, U = sort(lamb, U)
    elif algo == "eigh":
        lamb, U = np.linalg.eigh(L.toarray())
    elif algo == "eigs":
        import scipy.sparse.linalg
        lamb, U = scipy.sparse.linalg.eigs(L, k=k, which="SM")
        lamb, U = sort(lamb, U)
    elif algo == "eigsh":
        import scipy.sparse.linalg
        lamb, U = scipy.sparse.linalg.eigsh(L, k=k, which="SM")
    else:
        raise ValueError(f"unknown algo {algo!r}")
    return lamb, U


def rescale_L(L, lmax=2):
    """``L~ = L / (lmax/2) - I`` (lib/graph.py:232-238), on a private copy.

    The float32 operations are the reference's (scale ``data`` by the
    float32-rounded reciprocal, then a scipy subtraction that prunes explicit
    zeros), so L~ is bit-identical.  Unlike the reference this never mutates
    the caller's L (lib/filter.py:65 does when lmax != 2).
    """
    L = scipy.sparse.csr_matrix(L, copy=True)
    I = scipy.sparse.identity(L.shape[0], format="csr", dtype=L.dtype)
    L /= lmax / 2
    return L - I


def canonical_csr(A):
    """(rowptr int32, col int32, val float32) in row-major sorted order -- the
    order ``tocoo`` + ``tf.sparse_reorder`` give at lib/graph_conv.py:150-153."""
    A = scipy.sparse.csr_matrix(A, copy=True)
    A.sum_duplicates()
    A.sort_indices()
    return (np.ascontiguousarray(A.indptr, dtype=np.int32),
            np.ascontiguousarray(A.indices, dtype=np.int32),
            np.ascontiguousarray(A.data, dtype=np.float32))
