#!/usr/bin/env python3
"""Time one gconv-LSTM h-step (config E graph, N = 128, H = 32) for K = 1..4:
the fused launch (cg_lstm_hconv_step) vs chebyshev5 + the pointwise kernel.
The K slope separates the per-order work (MFMA + SpMM) from the fixed part
(prologue, epilogue).  python scripts/lstm_step_sweep.py"""
import json
import os
import sys

import numpy as np
import scipy.sparse
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cnn_graph_amd import ops  # noqa: E402
from cnn_graph_amd.plan import ChebPlan  # noqa: E402


def ev_us(fn, reps=20, rounds=5):
    vals = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        vals.append(e0.elapsed_time(e1) / reps * 1e3)
    return round(float(np.median(vals)), 1)


def main():
    dev = torch.device("cuda", 0)
    with np.load(os.path.join(ROOT, "tests", "golden", "golden_E.npz"), allow_pickle=False) as z:
        M = int(z["M"])
        Lt = scipy.sparse.csr_matrix((z["Lt_val"], z["Lt_col"], z["Lt_rowptr"]), shape=(M, M))
    plan = ChebPlan(Lt, device=0)
    N, H = 128, 32
    g = torch.Generator(device=dev)
    g.manual_seed(0)
    h = torch.randn((N, M, H), device=dev, generator=g) * 0.5
    c = torch.randn((N, M, H), device=dev, generator=g) * 0.5
    gx = torch.randn((N, M, 4 * H), device=dev, generator=g) * 0.5
    b = torch.randn((4 * H,), device=dev, generator=g) * 0.1
    out = {}
    for K in (1, 2, 3, 4):
        Wh = torch.randn((K * H, 4 * H), device=dev, generator=g) * 0.1
        co, ho, act = (torch.empty((N, M, H), device=dev), torch.empty((N, M, H), device=dev),
                       torch.empty((N, M, 4 * H), device=dev))
        planes = torch.empty((max(K - 1, 1), N * M, H), device=dev)
        basis = torch.empty((N * M, H * K), device=dev)
        gh = torch.empty((N, M, 4 * H), device=dev)

        def fused():
            ops.lstm_hconv_step(plan, h, c, gx, Wh, b, K, out_c=co, out_h=ho, out_act=act,
                                planes=planes[0], plane_stride=N * M * H)

        def unfused():
            ops.cheb_forward(plan, h, Wh, K, out_basis=basis, out_y=gh)
            ops.lstm_cell_forward(gx, gh, b, c, H, out_c=co, out_h=ho, out_act=act)

        fused()
        unfused()
        torch.cuda.synchronize()
        out[f"K{K}"] = {"fused_us": ev_us(fused), "unfused_us": ev_us(unfused)}
    print(json.dumps({"N": N, "M": M, "H": H, "steps": out}, indent=1))


if __name__ == "__main__":
    main()
