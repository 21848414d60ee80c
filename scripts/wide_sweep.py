#!/usr/bin/env python3
"""Wide-column step geometry sweep on config C1 (ablation build, CG_LIB_PATH):
column groups G (8 = one per XCD, 1 = none) x floats per lane (pl), timing
the forward (4 wide steps + re-layouts) -- results are unchanged by both.

  make debug && python scripts/wide_sweep.py
"""
import ctypes
import json
import os
import sys

import numpy as np
import scipy.sparse
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("CG_LIB_PATH", os.path.join(ROOT, "scripts", "_debug", "libcheb_mi355_debug.so"))
from cnn_graph_amd import _lib, ops  # noqa: E402
from cnn_graph_amd.plan import ChebPlan  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    with np.load(os.path.join(ROOT, "tests", "golden", "golden_C.npz"), allow_pickle=False) as z:
        M = int(z["M"])
        Lt = scipy.sparse.csr_matrix((z["Lt_val"], z["Lt_col"], z["Lt_rowptr"]), shape=(M, M))
    N, Fin, K, Fout = 128, 1, 5, 32
    h = _lib.lib()
    h.cg_debug_set_param.argtypes = [ctypes.c_int, ctypes.c_int]
    x = torch.rand((N, M, Fin), device=dev)
    W = torch.randn((Fin * K, Fout), device=dev) * 0.1
    dy = torch.randn((N, M, Fout), device=dev)
    ref = None
    out = {}
    for G in (8, 4, 2, 1):
        for pl in (4, 2, 1):
            h.cg_debug_set_param(0, G)
            h.cg_debug_set_param(1, pl)
            plan = ChebPlan(Lt, device=0)
            r = ops.ChebRunner(plan, N, Fin, K, Fout, dev)
            r.forward(x, W)
            r.backward(dy, W)
            torch.cuda.synchronize()
            same = True
            if ref is None:
                ref = (r.basis.clone(), r.dx.clone())
            else:
                same = bool(torch.equal(ref[0], r.basis) and torch.equal(ref[1], r.dx))
            vals_f, vals_b = [], []
            for _ in range(5):
                e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                e0.record()
                for _ in range(10):
                    r.forward(x, W)
                e1.record()
                for _ in range(10):
                    r.backward(dy, W)
                e2.record()
                torch.cuda.synchronize()
                vals_f.append(e0.elapsed_time(e1) / 10 * 1e3)
                vals_b.append(e1.elapsed_time(e2) / 10 * 1e3)
            out[f"G{G}_pl{pl}"] = {"fwd_us": round(float(np.median(vals_f)), 1),
                                   "bwd_us": round(float(np.median(vals_b)), 1), "same": same}
    h.cg_debug_set_param(0, -1)
    h.cg_debug_set_param(1, -1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
