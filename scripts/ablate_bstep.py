#!/usr/bin/env python3
"""Timing ablations + phase stamps of the one-launch gconv-LSTM BPTT step
(k_lstm_bstep, config E: N = 128, M = 1024, H = 32, K = 3) on the DEBUG build
(`make debug`, loaded through CG_LIB_PATH; outputs are garbage when a flag is
set -- timing only).  Flags (bits 16.. of cg_debug_set_flags): 1 no MFMA
(D_k), 2 no phase-A loads / gate math (dpre = 0), 4 no reverse recurrence.
Phase stamps (thread 0 of every workgroup, 100 MHz wall clock), us from the
workgroup's start: prologue (W, L~^T staged) done, phase A (dpre + D_k) done,
recurrence done, dh_prev stored -- median over the 256 workgroups, plus the
spread of the workgroups' start times."""
import ctypes
import json
import os
import sys

import numpy as np
import scipy.sparse
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("CG_LIB_PATH", os.path.join(ROOT, "scripts", "dbg", "libcheb_mi355_debug.so"))
from cnn_graph_amd import _lib, ops  # noqa: E402
from cnn_graph_amd.plan import ChebPlan  # noqa: E402

SETS = {"full": 0, "no_stores": 8, "no_mfma_stores": 9, "no_mfma": 1, "no_loads": 2, "no_rec": 4,
        "no_mfma_loads": 3,
        "only_rec": 3, "only_loads": 5, "only_mfma": 6, "nothing": 7}


def main():
    dev = torch.device("cuda", 0)
    with np.load(os.path.join(ROOT, "tests", "golden", "golden_E.npz"), allow_pickle=False) as z:
        M = int(z["M"])
        Lt = scipy.sparse.csr_matrix((z["Lt_val"], z["Lt_col"], z["Lt_rowptr"]), shape=(M, M))
    plan = ChebPlan(Lt, device=0)
    N, H, K = 128, 32, 3
    R = N * M
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    act = torch.rand((R, 4 * H), device=dev, generator=g) * 0.5
    cp, co, dh, dhr, dc = (torch.randn((R, H), device=dev, generator=g) for _ in range(5))
    Wh = torch.randn((K * H, 4 * H), device=dev, generator=g) * 0.1
    dpre = torch.empty((R, 4 * H), device=dev)
    dhp = torch.empty((R, H), device=dev)
    h = _lib.lib()
    h.cg_debug_set_flags.argtypes = [ctypes.c_int]
    h.cg_debug_set_ts.argtypes = [ctypes.c_void_p]

    def run():
        ops.lstm_bwd_step(plan, dh, dhr, dc, act, cp, co, Wh, K, out_dpre=dpre, out_dh_prev=dhp,
                          act_unit_major=True)

    out = {}
    buf = torch.zeros((2 * N, 8), dtype=torch.int64, device=dev)
    for rnd in range(3):
        for name, fl in SETS.items():
            h.cg_debug_set_flags(fl << 16)
            run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                run()
            e1.record()
            torch.cuda.synchronize()
            out.setdefault(name, {"us": []})["us"].append(e0.elapsed_time(e1) * 100)
            if rnd == 0:
                buf.zero_()
                h.cg_debug_set_ts(buf.data_ptr())
                run()
                torch.cuda.synchronize()
                h.cg_debug_set_ts(None)
                ts = buf.cpu().numpy().astype(np.float64)
                d = (ts[:, 1:5] - ts[:, :1]) * 0.01
                out[name]["phase_us"] = [round(float(np.median(d[:, i])), 2) for i in range(4)]
                st = (ts[:, 0] - ts[:, 0].min()) * 0.01
                out[name]["start_spread_us"] = [round(float(np.percentile(st, p)), 2) for p in (50, 90, 100)]
    h.cg_debug_set_flags(0)
    for name, v in out.items():
        v["us"] = round(float(np.median(v["us"])), 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
