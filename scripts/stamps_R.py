#!/usr/bin/env python3
"""Phase stamps of config R's hidden-layer filter kernels (M = 1024, N = 100,
Fin = Fout = 32, K = 20, planes layout) on the DEBUG build (CG_LIB_PATH):
k_grp16_fwd (0 start, 2 recurrence + contraction done, 3 y stored) and
k_grp_clen_dy (0 start, 1 prologue done, 2..6 order groups done, 7 dx stored).
Per kernel: median us of each stamp from the workgroup's own start, and the
distribution of workgroup start times (residency rounds), plus the HIP-event
time of 20 calls.  An optional argument sets k_grp16_fwd's ablation flags
(debug byte 24-31; k_grp16_fwd: 1 no MFMA, 2 no SpMM, 4 no plane stores;
k_grp_clen_dy: 1 no D-tile MFMAs, 2 no SpMM, 4 no dy loads, 8 no hand-over;
outputs garbage, times only) for the named call.
  python3 scripts/stamps_R.py [FLAGS [fwd|bwd]]"""
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


def stamps(buf, n_wg):
    ts = buf[:n_wg].cpu().numpy().astype(np.float64)
    ok = ts[:, 0] > 0
    ts = ts[ok]
    t0 = ts[:, 0]
    rel = {}
    for sl in range(1, 8):
        v = ts[:, sl]
        m = v > 0
        if m.any():
            rel[sl] = round(float(np.median((v[m] - t0[m]) * 0.01)), 2)
    st = (t0 - t0.min()) * 0.01
    end = max(ts[:, s].max() for s in range(8))
    return {"n_wg": int(ok.sum()), "phase_us": rel,
            "start_us_p50_p90_max": [round(float(np.percentile(st, p)), 1) for p in (50, 90, 100)],
            "span_us": round(float((end - t0.min()) * 0.01), 1)}


def main():
    with np.load(os.path.join(ROOT, "tests", "golden", "golden_E.npz"), allow_pickle=False) as z:
        M = int(z["M"])
        Lt = scipy.sparse.csr_matrix((z["Lt_val"], z["Lt_col"], z["Lt_rowptr"]), shape=(M, M))
    dev = torch.device("cuda", 0)
    plan = ChebPlan(Lt, device=0, path="stream")
    N, Fin, K, Fout = 100, 32, 20, 32
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    x = torch.rand((N, M, Fin), device=dev, generator=g)
    W = torch.randn((Fin * K, Fout), device=dev, generator=g) * 0.1
    dy = torch.randn((N, M, Fout), device=dev, generator=g)
    r = ops.ChebRunner(plan, N, Fin, K, Fout, dev, basis_layout="planes")
    h = _lib.lib()
    h.cg_debug_set_ts.argtypes = [ctypes.c_void_p]
    out = {}
    flags = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    which = sys.argv[2] if len(sys.argv) > 2 else "fwd"  # the call the flags apply to
    h.cg_debug_set_flags.argtypes = [ctypes.c_int]
    if flags:
        h.cg_debug_set_flags(flags << 24)
        out["flags"] = flags
    for name, fn in (("fwd", lambda: r.forward(x, W)), ("bwd", lambda: r.backward(dy, W))):
        if flags and name != which:
            continue
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        buf = torch.zeros((1024, 8), dtype=torch.int64, device=dev)
        h.cg_debug_set_ts(buf.data_ptr())
        fn()
        torch.cuda.synchronize()
        h.cg_debug_set_ts(None)
        out[name] = {"call_us": round(e0.elapsed_time(e1) / 20 * 1e3, 1), **stamps(buf, 1024)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
