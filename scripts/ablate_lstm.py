#!/usr/bin/env python3
"""Timing ablations + phase stamps of the one-launch gconv-LSTM layer forward
(k_lstm_seq, config E: N = 128, M = 1024, T = 12, H = 32, K = 3) on the DEBUG
build (`make debug`, loaded through CG_LIB_PATH; outputs are garbage when a
flag is set -- timing only).  Flags (bits 16.. of cg_debug_set_flags): 1 no
MFMA, 2 no SpMM, 4 no gate math, 8 no partner wait, 16 no gx / c loads,
32 no plane stores, 64 no act stores, 128 no c stores, 256 no h stores.  Phase stamps (step 1, thread 0 of every workgroup, 100 MHz):
step start, own quarters done, partner wait done, all quarters done, epilogue +
flag done -- median over workgroups, us from the step start."""
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

SETS = {"full": 0, "no_mfma": 1, "no_spmm": 2, "no_gate_math": 4, "no_wait": 8, "no_loads": 16,
        "no_planes": 32, "no_mfma_spmm": 3, "only_epilogue": 1 | 2 | 32, "nothing": 63,
        "no_act": 64, "no_act_c": 64 | 128, "no_stores": 64 | 128 | 256 | 32,
        "nothing_but_stores": 1 | 2 | 4 | 8 | 16}
XSETS = ("full", "no_loads", "nothing", "no_act", "no_act_c", "no_stores", "no_wait",
         "no_mfma_spmm", "nothing_but_stores")


def main():
    dev = torch.device("cuda", 0)
    with np.load(os.path.join(ROOT, "tests", "golden", "golden_E.npz"), allow_pickle=False) as z:
        M = int(z["M"])
        Lt = scipy.sparse.csr_matrix((z["Lt_val"], z["Lt_col"], z["Lt_rowptr"]), shape=(M, M))
    plan = ChebPlan(Lt, device=0)
    T, N, H, K = 12, 128, 32, 3
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    gx = torch.randn((T, N, M, 4 * H), device=dev, generator=g) * 0.3
    Wh = torch.randn((K * H, 4 * H), device=dev, generator=g) * 0.1
    b = torch.randn((4 * H,), device=dev, generator=g) * 0.1
    hs = torch.empty((T, N, M, H), device=dev)
    cs = torch.empty_like(hs)
    act = torch.empty((T, N, M, 4 * H), device=dev)
    planes = torch.empty((K - 1, T, N * M, H), device=dev)
    h = _lib.lib()
    h.cg_debug_set_flags.argtypes = [ctypes.c_int]
    h.cg_debug_set_ts.argtypes = [ctypes.c_void_p]

    Fin = 2
    xs = torch.rand((T, N, M, Fin), device=dev, generator=g)
    Wx = torch.randn((K * Fin, 4 * H), device=dev, generator=g) * 0.1
    xpl = torch.empty((K, T * N * M, Fin), device=dev)
    mode = {"x": False}

    def run():
        if mode["x"]:
            ops.lstm_seq_forward_x(plan, xs, Wx, Wh, b, K, out_hs=hs, out_cs=cs, out_act=act,
                                   planes=planes[0], plane_stride=T * N * M * H, xplanes=xpl)
        else:
            ops.lstm_seq_forward(plan, gx, Wh, b, K, T, N, out_hs=hs, out_cs=cs, out_act=act,
                                 planes=planes[0], plane_stride=T * N * M * H)

    out = {}
    buf = torch.zeros((256, 8), dtype=torch.int64, device=dev)
    sets = [(nm, fl, False) for nm, fl in SETS.items()] + \
        [("x_" + nm, fl, True) for nm, fl in SETS.items() if nm in XSETS]
    for rnd in range(3):
        for name, fl, xm in sets:
            mode["x"] = xm
            h.cg_debug_set_flags(fl << 16)
            run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                run()
            e1.record()
            torch.cuda.synchronize()
            out.setdefault(name, {"ms": []})["ms"].append(e0.elapsed_time(e1) / 5)
            if rnd == 0:
                buf.zero_()
                h.cg_debug_set_ts(buf.data_ptr())
                run()
                torch.cuda.synchronize()
                h.cg_debug_set_ts(None)
                ts = buf.cpu().numpy().astype(np.float64)
                d = (ts[:, 1:5] - ts[:, :1]) * 0.01
                out[name]["step1_us"] = [round(float(np.median(d[:, i])), 2) for i in range(4)]
    h.cg_debug_set_flags(0)
    for name, v in out.items():
        v["ms"] = round(float(np.median(v["ms"])), 4)
        v["per_step_us"] = round(v["ms"] * 1e3 / T, 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
