#!/usr/bin/env python3
"""Diagnostic: per-step s_memtime stamps of the resident forward (block 0,
wave 0), written into y by the dbg&32 build path.  Timing-only; outputs wrong."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from cnn_graph_amd import _lib, ops  # noqa: E402
from cnn_graph_amd.plan import ChebPlan  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    L, fake = bench.load_config_b()
    K, Fin, Fout, N = 25, 1, 32, 256
    plan = ChebPlan.from_laplacian(L, 2, 0, path="resident")
    x = torch.rand((N, plan.M, Fin), device=dev)
    W = torch.randn((K, Fout), device=dev) * 0.1
    r = ops.ChebRunner(plan, N, Fin, K, Fout, dev)
    h = _lib.lib()
    out = {}
    for name, f in (("full", 32), ("no_spmm", 33), ("no_store_mfma", 32 | 2 | 4), ("nothing", 32 | 15)):
        h.cg_debug_set_flags(f)
        for _ in range(20):
            r.forward(x, W)
        torch.cuda.synchronize()
        y = r.y.reshape(-1)[: 2 * K].cpu().numpy().astype(np.float64)
        pair = [y[2 * k] - y[2 * k - 1] if k > 1 else y[2] for k in range(1, K)]  # barrier+mfma_pair
        spmm = [y[2 * k + 1] - y[2 * k] for k in range(1, K)]
        out[name] = {"total_cycles": y[0], "per_step_cycles": round(y[0] / (K - 1), 1),
                     "spmm_cycles_med": float(np.median(spmm)),
                     "barrier_pair_cycles_med": float(np.median(pair[1:])),
                     "spmm_each": [round(v) for v in spmm[:6]], "pair_each": [round(v) for v in pair[:6]]}
    h.cg_debug_set_flags(0)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
