#!/usr/bin/env python3
"""Would a channel-sliced XCD mapping shrink config D's SpMM gather traffic?


CPU model of one k_cheb_step pass over one sample's slab T_{k-1}[n] (M = 2^18
vertices, Fin = 64 fp32 = 256 B per vertex row, 67 MB per sample) on the 8
XCDs, each with a 4 MiB L2 modelled as a fully associative LRU over 128-B
lines (32 768 of them); every L2 miss is one 128-B line from the Infinity
Cache / HBM (the fabric traffic the PMC counts).  Rows are processed in the
kernel's order (longest first: the plan's degree-sorted row order on skewed
graphs) and each row gathers its CSR columns in CSR order.

  current    all 8 XCDs on one sample, 16-row blocks dealt round-robin to the
             XCDs; each gather reads the whole 256-B row = its 2 lines
  slice8     XCD x owns channels 8x .. 8x+7 of EVERY row of the sample (slab
             layout unchanged, [M][64]): a gather reads 32 B = one line (the
             line holds 4 XCDs' slices); every XCD walks all rows
  slice8_pl  the same with the slab re-laid as 8 channel planes [8][M][8]
             (32 B per row, 4 rows per line): an XCD's slab is 8.4 MB
  slice16_pl 16-channel planes [4][M][16] (64 B per row, 2 rows per line),
             XCD pairs on two samples at once (per sample: 4 slice streams)

Output: one JSON line per scheme: L2 hit rate of the gathers and the fabric
bytes per step per sample (misses x 128 B summed over the streams of one
sample), against the current mapping's.
"""
import json
import os
import sys
import time
from collections import OrderedDict

import numpy as np
import scipy.sparse

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))

XCDS = 8
L2_LINES = (4 << 20) // 128
ROWS_PER_BLOCK = 16


def lru_stream(indptr, indices, rows, line_of, lines_per_gather):
    """(hits, misses) of one XCD's gather stream: the CSR columns of `rows`
    in order; a gather of column c touches lines line_of(c) .. + lines_per_gather-1."""
    c = OrderedDict()
    hits = misses = 0
    for r in rows:
        for col in indices[indptr[r]:indptr[r + 1]]:
            base = line_of(int(col))
            for q in range(lines_per_gather):
                ln = base + q
                if ln in c:
                    hits += 1
                    c.move_to_end(ln)
                else:
                    misses += 1
                    c[ln] = None
                    if len(c) > L2_LINES:
                        c.popitem(last=False)
    return hits, misses


def main():
    from synth_graphs import chung_lu
    t0 = time.time()
    A = scipy.sparse.csr_matrix(chung_lu())
    M = A.shape[0]
    indptr, indices = A.indptr, A.indices
    deg = np.diff(indptr)
    order = np.argsort(-deg, kind="stable")  # the plan's longest-first row order
    out = []
    # current: blocks of 16 rows round-robin over the XCDs, 2 lines per gather
    h = m = 0
    for x in range(XCDS):
        blocks = [order[b:b + ROWS_PER_BLOCK] for b in range(x * ROWS_PER_BLOCK, M, XCDS * ROWS_PER_BLOCK)]
        rows = np.concatenate(blocks)
        hh, mm = lru_stream(indptr, indices, rows, lambda c: 2 * c, 2)
        h, m = h + hh, m + mm
    cur = m * 128
    out.append(("current", h / (h + m), cur, 8))
    # slice8: every XCD walks all rows, one line per gather (line = row's half)
    hh, mm = lru_stream(indptr, indices, order, lambda c: c, 1)
    out.append(("slice8", hh / (hh + mm), 8 * mm * 128, 8))
    # slice8_pl: [8][M][8]: 4 rows per line
    hh, mm = lru_stream(indptr, indices, order, lambda c: c // 4, 1)
    out.append(("slice8_pl", hh / (hh + mm), 8 * mm * 128, 8))
    # slice16_pl: [4][M][16]: 2 rows per line, 4 streams per sample
    hh, mm = lru_stream(indptr, indices, order, lambda c: c // 2, 1)
    out.append(("slice16_pl", hh / (hh + mm), 4 * mm * 128, 4))
    for name, hit, fabric, streams in out:
        print(json.dumps({"scheme": name, "l2_hit_rate": round(hit, 4),
                          "fabric_MB_per_step_per_sample": round(fabric / 1e6, 1),
                          "vs_current": round(fabric / cur, 3), "streams_per_sample": streams,
                          "gathers": int(indptr[-1]), "elapsed_s": round(time.time() - t0, 1)}),
              flush=True)


if __name__ == "__main__":
    main()
