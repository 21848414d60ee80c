#!/usr/bin/env python3
"""Would relabelling config D's vertices make its SpMM gathers cache-local?

CPU model of the streaming Chebyshev step's gather stream (k_cheb_step, Fin =
64: one vertex row of the gathered slab T_{k-1}[n] = 256 B = two whole 128-B
lines, so two vertices never share a line -- a relabelling can only change
TEMPORAL reuse, i.e. which rows are processed close together).  Rows are
processed in label order in blocks of ROWS_PER_BLOCK dealt round-robin to the
8 XCDs (the all-XCDs-on-one-sample mapping of the large-slab path, DESIGN.md
§streaming path 2); each XCD's 4 MB L2 is modelled as an LRU over vertex
rows (16 384 of them).  Every L2 miss is a 256-B read from the Infinity Cache
(the 67 MB slab stays there).  Orderings: the generator's random ids (what
the benchmark runs), reverse Cuthill-McKee, degree-descending, and a BFS
order -- each applied to rows AND columns (a symmetric relabelling; the CSR
entries of a row can keep their original order, so the basis would stay
bit-exact).

Output: one JSON line per ordering with the L2 hit rate of the gathers and
the gathered bytes that leave L2 per step per sample.
"""
import json
import os
import sys
import time
from collections import OrderedDict

import numpy as np
import scipy.sparse
import scipy.sparse.csgraph as csg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))

ROWS_PER_BLOCK = 16     # k_cheb_step at Fin = 64: 16 lanes per row, 256 threads
XCDS = 8
L2_ROWS = (4 << 20) // 256


def simulate(A, order, contiguous=False):
    """L2 hits / gathers of one SpMM pass with rows processed in `order`;
    contiguous: XCD x takes the x-th eighth of the order (instead of blocks
    dealt round-robin), so a locality-preserving order keeps each XCD's rows
    together."""
    caches = [OrderedDict() for _ in range(XCDS)]
    hits = total = 0
    indptr, indices = A.indptr, A.indices
    n = len(order)
    for p, r in enumerate(order):
        c = caches[p * XCDS // n if contiguous else (p // ROWS_PER_BLOCK) % XCDS]
        for col in indices[indptr[r]:indptr[r + 1]]:
            total += 1
            if col in c:
                hits += 1
                c.move_to_end(col)
            else:
                c[col] = None
                if len(c) > L2_ROWS:
                    c.popitem(last=False)
    return hits, total


def main():
    from synth_graphs import chung_lu
    t0 = time.time()
    W = chung_lu()
    A = scipy.sparse.csr_matrix(W)
    M = A.shape[0]
    deg = np.diff(A.indptr)
    orders = {
        "random_ids (benchmarked)": np.arange(M),
        "rcm": csg.reverse_cuthill_mckee(A, symmetric_mode=True),
        "degree_desc": np.argsort(-deg, kind="stable"),
        "bfs": csg.breadth_first_order(A, int(np.argmax(deg)), directed=False,
                                       return_predecessors=False),
    }
    for name, order in orders.items():
        order = np.asarray(order)
        if order.size < M:  # BFS from one vertex: unreached vertices appended
            seen = np.zeros(M, bool)
            seen[order] = True
            order = np.concatenate([order, np.flatnonzero(~seen)])
        # a symmetric relabelling: new label i = old vertex order[i]; the row
        # processed at position p is order[p] and its neighbours keep their
        # identity, so the gather stream is the old columns in this row order
        for contiguous in ((False, True) if name in ("rcm", "bfs") else (False,)):
            hits, total = simulate(A, order, contiguous)
            print(json.dumps({"ordering": name, "xcd_rows": "contiguous" if contiguous else "round_robin",
                              "gathers": total, "l2_hit_rate": round(hits / total, 4),
                              "l2_miss_bytes_per_step_per_sample_MB": round((total - hits) * 256 / 1e6, 1),
                              "gathered_bytes_MB": round(total * 256 / 1e6, 1),
                              "elapsed_s": round(time.time() - t0, 1)}), flush=True)


if __name__ == "__main__":
    main()
