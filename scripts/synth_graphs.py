"""Synthetic graphs for the large configurations of SURVEY.md §8d.

  config D: Chung-Lu power-law graph, M = 2**18 vertices, nnz(W) ~= 4.19 M,
            symmetrised with max(W, W^T) like lib/graph.py:77-78 (adjacency),
            edge weights U(0, 1], vertex ids randomly permuted (no locality
            artefact of the generator), seeded -> deterministic.
Used by bench.py's --config D and by the large-graph GPU tests; not part of
the shipped filter path.
"""
from __future__ import annotations

import numpy as np
import scipy.sparse


def chung_lu(M=1 << 18, avg_deg=16.0, gamma=2.5, max_deg=1024, seed=2017):
    """Symmetric weighted adjacency W (csr, float32) of a Chung-Lu graph whose
    expected degrees follow a power law with exponent ``gamma`` (capped at
    ``max_deg``) and average ~``avg_deg``."""
    rng = np.random.default_rng(seed)
    w = (np.arange(M, dtype=np.float64) + 10.0) ** (-1.0 / (gamma - 1.0))
    w *= avg_deg * M / w.sum()
    w = np.minimum(w, max_deg)
    w *= avg_deg * M / w.sum()
    p = w / w.sum()
    E = int(round(avg_deg * M / 2))
    u = rng.choice(M, size=E, p=p)
    v = rng.choice(M, size=E, p=p)
    keep = u != v
    u, v = u[keep], v[keep]
    val = (1.0 - rng.random(u.size)).astype(np.float32)          # U(0, 1]
    perm = rng.permutation(M)                                     # random vertex ids
    u, v = perm[u], perm[v]
    W = scipy.sparse.coo_matrix((val, (u, v)), shape=(M, M)).tocsr()
    W.sum_duplicates()
    bigger = W.T > W                                              # lib/graph.py:77-78
    W = W - W.multiply(bigger) + W.T.multiply(bigger)
    W = scipy.sparse.csr_matrix(W, dtype=np.float32)
    W.eliminate_zeros()
    W.sort_indices()
    return W


def config_d_laplacian(seed=2017):
    """Normalized Laplacian of the config-D graph (lib/graph.py:117-136)."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from cnn_graph_amd.graph import laplacian
    return laplacian(chung_lu(seed=seed), normalized=True)


if __name__ == "__main__":
    import time
    t = time.time()
    W = chung_lu()
    deg = np.diff(W.indptr)
    print(f"M={W.shape[0]} nnz={W.nnz} max_row={deg.max()} mean={deg.mean():.2f} "
          f"p99={np.percentile(deg, 99):.0f} isolated={(deg == 0).sum()} {time.time() - t:.1f}s")
