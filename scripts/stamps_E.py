#!/usr/bin/env python3
"""Phase stamps of config E's layer forward on the DEBUG build (CG_LIB_PATH):
k_lstm_seq (default) or k_lstm_seq2 (CG_SEQ_V=2), step 1 of the first sample of
every pair: 0 step start, 1 own quarters' recurrence done (seq2: phase 1),
2 partner wait done, 3 contraction + gates done (seq2: phase 2) [k_lstm_seq:
3 all quarters contracted, 4 epilogue done].  Median over workgroups, us from
the step start; plus the HIP-event time of the layer forward.  An optional
argument sets the debug build's ablation flags for the whole run (k_lstm_seq2
phase 2: 1 no MFMA, 2 no SpMM, 4 linear gates, 16 no gx / c loads, 64 no
act stores, 128 no c stores; outputs are garbage, times only); they go to the
sequence kernels' byte of the debug flags (bits 16-23).
  python3 scripts/stamps_E.py [FLAGS]"""
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


def main():
    dev = torch.device("cuda", 0)
    with np.load(os.path.join(ROOT, "tests", "golden", "golden_E.npz"), allow_pickle=False) as z:
        M = int(z["M"])
        Lt = scipy.sparse.csr_matrix((z["Lt_val"], z["Lt_col"], z["Lt_rowptr"]), shape=(M, M))
    plan = ChebPlan(Lt, device=0)
    T, N, H, K, Fin = 12, 128, 32, 3, 2
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    xs = torch.rand((T, N, M, Fin), device=dev, generator=g)
    Wx = torch.randn((K * Fin, 4 * H), device=dev, generator=g) * 0.1
    Wh = torch.randn((K * H, 4 * H), device=dev, generator=g) * 0.1
    b = torch.randn((4 * H,), device=dev, generator=g) * 0.1
    R = T * N * M
    hs = torch.empty((T, N, M, H), device=dev)
    cs = torch.empty_like(hs)
    act = torch.empty((R, 4 * H), device=dev)
    planes = torch.empty((K - 1, R, H), device=dev)
    xpl = torch.empty((K, R, Fin), device=dev)

    def run():
        ops.lstm_seq_forward_x(plan, xs, Wx, Wh, b, K, out_hs=hs, out_cs=cs, out_act=act,
                               planes=planes[0], plane_stride=R * H, xplanes=xpl)

    h = _lib.lib()
    h.cg_debug_set_ts.argtypes = [ctypes.c_void_p]
    flags = int(sys.argv[1]) if len(sys.argv) > 1 else 0
    h.cg_debug_set_flags.argtypes = [ctypes.c_int]
    h.cg_debug_set_flags(flags << 16)
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        run()
    e1.record()
    torch.cuda.synchronize()
    buf = torch.zeros((256, 8), dtype=torch.int64, device=dev)
    h.cg_debug_set_ts(buf.data_ptr())
    run()
    torch.cuda.synchronize()
    h.cg_debug_set_ts(None)
    ts = buf.cpu().numpy().astype(np.float64)
    d = (ts[:, 1:5] - ts[:, :1]) * 0.01
    h.cg_debug_set_flags(0)
    print(json.dumps({"kernel": "k_lstm_seq2" if os.environ.get("CG_SEQ_V") == "2" else "k_lstm_seq",
                      "flags": flags,
                      "layer_fwd_ms": round(e0.elapsed_time(e1) / 5, 4),
                      "step1_us": [round(float(np.median(d[:, i])), 2) for i in range(4)]}))


if __name__ == "__main__":
    main()
