#!/usr/bin/env python3
"""Per-workgroup phase timeline of the fast resident kernels on config B
(N = 256): thread 0 of every workgroup stamps the wall clock (s_memrealtime,
100 MHz) at the phase boundaries (CG_TS in cheb_fast_kern.h; ablation build
only).  Prints, per phase boundary, the median / max over workgroups of the
time since the earliest workgroup start, next to the HIP-event kernel time.

  make debug && python scripts/phase_ts.py
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("CG_LIB_PATH", os.path.join(ROOT, "scripts", "_debug", "libcheb_mi355_debug.so"))
import bench  # noqa: E402
from cnn_graph_amd import _lib, ops  # noqa: E402
from cnn_graph_amd.plan import ChebPlan  # noqa: E402

FWD = ["entry", "prologue", "recurrence", "y_issued", "end"]
BWD = ["entry", "prologue", "phase_a", "rows_loaded", "recurrence", "end"]
TICK_US = 0.01  # 100 MHz


def timeline(ts, names):
    t0 = ts[:, 0].min()
    out = {}
    for s, nm in enumerate(names):
        v = (ts[:, s] - t0) * TICK_US
        out[nm] = [round(float(np.median(v)), 2), round(float(v.max()), 2)]
    return out


def main():
    dev = torch.device("cuda", 0)
    L, fake = bench.load_config_b()
    K, Fin, Fout, N = 25, 1, 32, 256
    plan = ChebPlan.from_laplacian(L, 2, 0)
    h = _lib.lib()
    h.cg_debug_set_ts.argtypes = [ctypes.c_void_p]
    x = torch.rand((N, plan.M, Fin), device=dev)
    W = torch.randn((K, Fout), device=dev) * 0.1
    dy = torch.randn((N, plan.M, Fout), device=dev)
    buf = torch.zeros((N, 8), dtype=torch.int64, device=dev)
    res = {}
    for layout in ("rows", "orders"):
        r = ops.ChebRunner(plan, N, Fin, K, Fout, dev, basis_layout=layout)
        for _ in range(5):
            r.forward(x, W)
            r.backward(dy, W)
        for name, fn, names in (("fwd", lambda: r.forward(x, W), FWD),
                                ("bwd", lambda: r.backward(dy, W), BWD)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
            lines = []
            for _ in range(5):
                buf.zero_()
                h.cg_debug_set_ts(buf.data_ptr())
                fn()
                torch.cuda.synchronize()
                h.cg_debug_set_ts(None)
                lines.append(timeline(buf.cpu().numpy(), names))
            med = {k: [round(float(np.median([ln[k][i] for ln in lines])), 2) for i in (0, 1)]
                   for k in names}
            res[f"{layout}:{name}"] = {"kernel_us": round(e0.elapsed_time(e1) / 20 * 1e3, 2),
                                       "phase_us_median_max": med}
    # backward ablations (rows layout; outputs wrong): the fused dW's MFMAs
    # or its operand loads skipped during the recurrence
    h.cg_debug_set_flags.argtypes = [ctypes.c_int]
    r = ops.ChebRunner(plan, N, Fin, K, Fout, dev, basis_layout="rows")
    for tag, flags in (("bwd_no_dw_mfma", 64 << 8), ("bwd_no_dw_load", 128 << 8),
                       ("bwd_no_dw_both", 192 << 8)):
        h.cg_debug_set_flags(flags)
        lines = []
        for _ in range(5):
            buf.zero_()
            h.cg_debug_set_ts(buf.data_ptr())
            r.backward(dy, W)
            torch.cuda.synchronize()
            h.cg_debug_set_ts(None)
            lines.append(timeline(buf.cpu().numpy(), BWD))
        h.cg_debug_set_flags(0)
        res[f"rows:{tag}"] = {"kernel_us": None, "phase_us_median_max": {
            k: [round(float(np.median([ln[k][i] for ln in lines])), 2) for i in (0, 1)] for k in BWD}}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
