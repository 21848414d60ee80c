#!/usr/bin/env python3
"""Phase timeline of cheb_fwd_fast on config B (N = 256) for the 1 024-thread
build (one row per lane) against the 512-thread build (two rows per lane,
CG_OPT_FAST_RPL = 2), packed or scalar sums (forward debug bit 1), in the
ablation build (CG_TS stamps: entry, prologue, recurrence, y issued, end; µs
from the first workgroup's start, median / max over workgroups), plus the
HIP-event kernel time of each.

  make debug DEBUG_LIB=scripts/dbglib/libcheb_mi355_debug.so && python scripts/rpl_stamps.py
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
os.environ.setdefault("CG_LIB_PATH", os.path.join(ROOT, "scripts", "dbglib", "libcheb_mi355_debug.so"))
import bench  # noqa: E402
from phase_ts import FWD, timeline  # noqa: E402
from cnn_graph_amd import _lib, ops  # noqa: E402
from cnn_graph_amd.plan import ChebPlan  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    L, fake = bench.load_config_b()
    K, Fin, Fout, N = 25, 1, 32, 256
    plan = ChebPlan.from_laplacian(L, 2, 0)
    h = _lib.lib()
    h.cg_debug_set_ts.argtypes = [ctypes.c_void_p]
    h.cg_debug_set_flags.argtypes = [ctypes.c_int]
    x = torch.rand((N, plan.M, Fin), device=dev)
    W = torch.randn((K, Fout), device=dev) * 0.1
    buf = torch.zeros((N, 8), dtype=torch.int64, device=dev)
    res = {}
    for layout in ("orders", "rows"):
        for tag, rpl, flags in (("rpl1", 1, 0), ("rpl2_packed", 2, 0), ("rpl2_scalar", 2, 1),
                                ("rpl1_no_mfma", 1, 4), ("rpl2_no_mfma", 2, 4)):
            _lib.set_option("fast_rpl", rpl)
            h.cg_debug_set_flags(flags)
            r = ops.ChebRunner(plan, N, Fin, K, Fout, dev, basis_layout=layout)
            for _ in range(20):
                r.forward(x, W)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(50):
                r.forward(x, W)
            e1.record()
            torch.cuda.synchronize()
            lines = []
            for _ in range(7):
                buf.zero_()
                h.cg_debug_set_ts(buf.data_ptr())
                r.forward(x, W)
                torch.cuda.synchronize()
                h.cg_debug_set_ts(None)
                lines.append(timeline(buf.cpu().numpy(), FWD))
            med = {k: [round(float(np.median([ln[k][i] for ln in lines])), 2) for i in (0, 1)] for k in FWD}
            res[f"{layout}:{tag}"] = {"kernel_us": round(e0.elapsed_time(e1) / 50 * 1e3, 2),
                                      "phase_us_median_max": med}
            h.cg_debug_set_flags(0)
    _lib.set_option("fast_rpl", 1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
