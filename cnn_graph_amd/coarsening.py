"""Graph coarsening for the pooled (multi-level) model -- lib/coarsening.py API.

``coarsen(A, levels)`` builds the Graclus hierarchy whose binary-tree vertex
order makes graph max-pooling a plain stride-p window (lib/graph_conv.py:201-209,
device kernel cg_maxpool_forward), and ``perm_data`` moves signals into that
order (device kernel cg_perm_gather via ``ops.perm_data``; the host function
here keeps the reference's NumPy signature).

The greedy matching (lib/coarsening.py:119-165) and the tree order
(:167-214) run natively in libcheb_mi355.so (cg_graclus_match_*,
cg_compute_perm) -- the reference's pure-Python loops take seconds at MNIST
size.  Everything that decides WHICH order those loops see is computed here
with the reference's own NumPy calls, because it is implementation-defined:

* the COO order of ``scipy.sparse.find`` followed by the *unstable*
  ``np.argsort(idx_row)`` (:82-86) permutes entries inside a row, and the
  matching breaks ties by that order;
* the level-0 visit order is ``np.random.permutation`` (:56, unseeded in the
  reference; pass ``rid`` to pin it) and later levels use the default-kind
  ``np.argsort`` of the degrees (:112-113), which has massive ties.

``rids`` (one visit order per level) may be injected to reproduce a recorded
run exactly (tests/golden/golden_B.npz records the reference's).
"""
from __future__ import annotations

import ctypes

import numpy as np
import scipy.sparse

from . import _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def metis_one_level(rr, cc, vv, rid, weights):
    """One level of Graclus matching (lib/coarsening.py:119-165) -> cluster_id.

    ``rr`` ascending row indices, ``cc``/``vv`` the matching columns/weights in
    the order the reference's ``metis`` produced them; ``rid`` the visit order;
    ``weights`` the per-vertex Graclus weights.  The pairing score is computed
    in the dtype of ``vv`` (float32 graphs: NumPy-2 float32 arithmetic)."""
    rr = np.ascontiguousarray(rr, np.int32)
    cc = np.ascontiguousarray(cc, np.int32)
    rid = np.ascontiguousarray(rid, np.int64)
    if np.asarray(vv).dtype == np.float64 or np.asarray(weights).dtype == np.float64:
        vv = np.ascontiguousarray(vv, np.float64)
        weights = np.ascontiguousarray(weights, np.float64)
        fn = "cg_graclus_match_f64"
    else:
        vv = np.ascontiguousarray(vv, np.float32)
        weights = np.ascontiguousarray(weights, np.float32)
        fn = "cg_graclus_match_f32"
    nnz = rr.shape[0]
    if nnz == 0:
        raise ValueError("metis_one_level: graph has no edges")
    N = int(rr[-1]) + 1
    if weights.shape[0] < N:
        raise ValueError("metis_one_level: weights shorter than the vertex count")
    cluster_id = np.zeros(N, np.int32)
    ncl = ctypes.c_int32(0)
    _lib.call(fn, nnz, _ptr(rr), _ptr(cc), _ptr(vv), int(rid.shape[0]), _ptr(rid), _ptr(weights),
              _ptr(cluster_id), ctypes.byref(ncl))
    return cluster_id


def metis(W, levels, rid=None, rids=None):
    """Coarsen ``W`` ``levels`` times (lib/coarsening.py:34-115).

    Returns (graphs, parents) like the reference.  ``rid``: level-0 visit order
    (default: ``np.random.permutation``, as the reference); ``rids``: a visit
    order per level, overriding both ``rid`` and the per-level argsort."""
    N = W.shape[0]
    if rids is not None:
        rids = list(rids)
        if len(rids) < levels:
            raise ValueError(f"rids has {len(rids)} visit orders for {levels} levels")
        rid = rids[0]
    elif rid is None:
        rid = np.random.permutation(range(N))
    parents = []
    degree = W.sum(axis=0) - W.diagonal()
    graphs = [W]
    for lvl in range(levels):
        weights = np.array(degree).squeeze()
        idx_row, idx_col, val = scipy.sparse.find(W)
        perm = np.argsort(idx_row)  # default (unstable) kind, as the reference
        rr, cc, vv = idx_row[perm], idx_col[perm], val[perm]
        cluster_id = metis_one_level(rr, cc, vv, rid, weights)
        parents.append(cluster_id)
        nrr, ncc = cluster_id[rr], cluster_id[cc]
        Nnew = int(cluster_id.max()) + 1
        W = scipy.sparse.csr_matrix((vv, (nrr, ncc)), shape=(Nnew, Nnew))
        W.eliminate_zeros()
        graphs.append(W)
        degree = W.sum(axis=0)
        if rids is not None and lvl + 1 < levels:
            rid = rids[lvl + 1]
        else:
            ss = np.array(W.sum(axis=0)).squeeze()
            rid = np.argsort(ss)
    return graphs, parents


def compute_perm(parents):
    """Binary-tree vertex orders, coarsest level first in the recursion, returned
    finest first (lib/coarsening.py:167-214).  Lists of int, like the reference."""
    if len(parents) == 0:
        return []
    par = [np.ascontiguousarray(p, np.int32) for p in parents]
    levels = len(par)
    n_last = int(par[-1].max()) + 1
    sizes = np.array([p.shape[0] for p in par] + [n_last], np.int32)
    cap = n_last * ((1 << (levels + 1)) - 1)
    out = np.empty(cap, np.int32)
    sizes_out = np.empty(levels + 1, np.int32)
    flat = np.ascontiguousarray(np.concatenate(par))
    _lib.call("cg_compute_perm", levels, _ptr(sizes), _ptr(flat), _ptr(out), cap, _ptr(sizes_out))
    res, o = [], 0
    for n in sizes_out:
        res.append(out[o:o + int(n)].tolist())
        o += int(n)
    return res


def perm_data(x, indices):
    """Host perm_data (lib/coarsening.py:219-240): N x M -> N x len(indices),
    fake vertices 0, float64 result like the reference's ``np.empty``.  The
    device version for training batches is ``cnn_graph_amd.ops.perm_data``."""
    if indices is None:
        return x
    N, M = x.shape
    idx = np.asarray(indices)
    if idx.shape[0] < M:
        raise ValueError("perm_data: fewer indices than vertices")
    out = np.zeros((N, idx.shape[0]))
    real = idx < M
    out[:, real] = x[:, idx[real]]
    return out


def perm_adjacency(A, indices):
    """Permute (and pad with isolated fake vertices) an adjacency matrix
    (lib/coarsening.py:243-270).  Returns COO like the reference."""
    if indices is None:
        return A
    M = A.shape[0]
    Mnew = len(indices)
    if Mnew < M:
        raise ValueError("perm_adjacency: fewer indices than vertices")
    A = A.tocoo()
    if Mnew > M:
        rows = scipy.sparse.coo_matrix((Mnew - M, M), dtype=np.float32)
        cols = scipy.sparse.coo_matrix((Mnew, Mnew - M), dtype=np.float32)
        A = scipy.sparse.vstack([A, rows])
        A = scipy.sparse.hstack([A, cols])
    perm = np.argsort(indices)
    A = A.tocoo()
    A.row = np.array(perm)[A.row]
    A.col = np.array(perm)[A.col]
    return A


def coarsen(A, levels, self_connections=False, rid=None, rids=None, verbose=True):
    """Graph hierarchy + level-0 data permutation (lib/coarsening.py:5-31).

    Returns (graphs, perm): ``graphs[i]`` the permuted CSR adjacency of level i
    (fake vertices isolated, diagonal removed unless ``self_connections``),
    ``perm`` the order to apply to signals with ``perm_data``."""
    graphs, parents = metis(A, levels, rid=rid, rids=rids)
    perms = compute_perm(parents)
    for i, G in enumerate(graphs):
        M = G.shape[0]
        if not self_connections:
            G = G.tocoo()
            G.setdiag(0)
        if i < levels:
            G = perm_adjacency(G, perms[i])
        G = G.tocsr()
        G.eliminate_zeros()
        graphs[i] = G
        Mnew = G.shape[0]
        if verbose:
            print(f"Layer {i}: M_{i} = |V| = {Mnew} nodes ({Mnew - M} added),"
                  f"|E| = {G.nnz // 2} edges")
    return graphs, perms[0] if levels > 0 else None
