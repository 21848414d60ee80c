#!/usr/bin/env python3
"""Timing ablations of the resident kernels (outputs are garbage when a flag is
set -- timing only).  Interleaved rounds in one process (guide §5.4 rule 24).
Runs on the DEBUG build of the library (`make debug`: the ablation switches
are compiled out of the release .so), loaded through CG_LIB_PATH.

  make debug && python scripts/ablate.py [--batch 256] [--reps 50] [--rounds 5]
"""
import argparse
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

# (cg_debug_set_flags value, plan variant): flag bits 0-7 forward kernel,
# 8-15 backward kernel, 22 skip dW, 23 skip slab reduce
FWD = {"full": (0, "auto"), "no_basis_store": (2, "auto"), "no_mfma": (4, "auto"),
       "no_y_store": (8, "auto"), "no_stores": (2 | 8, "auto"), "only_spmm": (2 | 4 | 8, "auto"),
       "prologue": (16, "auto"), "classic": (0, "classic"), "ring_tkm2": (32, "auto")}
BWD = {"full": (0, "auto"), "no_phaseA": (2 << 8, "auto"), "prologue": (16 << 8, "auto"),
       "no_fused_dw": (0, "unfused_dw"), "no_dw": (1 << 22, "unfused_dw"),
       "no_reduce": (1 << 23, "auto"), "classic": (0, "classic"), "ring_gkp2": (32 << 8, "auto")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--path", default="resident")
    ap.add_argument("--layout", default="rows", choices=["rows", "orders"],
                    help="basis layout of the default-variant runner")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    L, fake = bench.load_config_b()
    K, Fin, Fout, N = 25, 1, 32, args.batch
    plan = ChebPlan.from_laplacian(L, 2, 0, path=args.path)
    M = plan.M
    x = torch.rand((N, M, Fin), device=dev)
    W = torch.randn((K, Fout), device=dev) * 0.1
    dy = torch.randn((N, M, Fout), device=dev)
    runners = {v: ops.ChebRunner(ChebPlan.from_laplacian(L, 2, 0, path=args.path, variant=v),
                                 N, Fin, K, Fout, dev,
                                 basis_layout=args.layout if v == "auto" else "rows")
               for v in ("auto", "classic", "unfused_dw")}
    r = runners["auto"]
    h = _lib.lib()
    h.cg_debug_set_flags.argtypes = [ctypes_int()]

    def t_fwd(r):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            r.forward(x, W)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.reps * 1e3

    def t_bwd(r):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            r.backward(dy, W)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.reps * 1e3

    res = {f"fwd:{k}": [] for k in FWD}
    res.update({f"bwd:{k}": [] for k in BWD})
    r.forward(x, W)
    for _ in range(args.rounds):
        for k, (f, v) in FWD.items():
            h.cg_debug_set_flags(f)
            res[f"fwd:{k}"].append(t_fwd(runners[v]))
        for k, (f, v) in BWD.items():
            runners[v].forward(x, W)
            h.cg_debug_set_flags(f)
            res[f"bwd:{k}"].append(t_bwd(runners[v]))
    h.cg_debug_set_flags(0)
    out = {k: round(float(np.median(v)), 2) for k, v in res.items()}
    # K sweep: per-step cost = slope of time vs K
    sweep = {}
    for Kx in (2, 7, 13, 25):
        Wx = torch.randn((Kx, Fout), device=dev) * 0.1
        rx = ops.ChebRunner(plan, N, Fin, Kx, Fout, dev, basis_layout=args.layout)
        for name, f in (("fwd_full", 0), ("fwd_only_spmm", FWD["only_spmm"][0]), ("bwd_full", 0),
                        ("bwd_no_dw", 1 << 22)):
            vals = []
            for _ in range(args.rounds):
                if name.startswith("fwd"):
                    h.cg_debug_set_flags(f)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(args.reps):
                        rx.forward(x, Wx)
                    e1.record()
                else:
                    h.cg_debug_set_flags(f)
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(args.reps):
                        rx.backward(dy, Wx)
                    e1.record()
                torch.cuda.synchronize()
                vals.append(e0.elapsed_time(e1) / args.reps * 1e3)
            sweep[f"K{Kx}:{name}"] = round(float(np.median(vals)), 2)
    h.cg_debug_set_flags(0)
    print(json.dumps({"batch": N, "path": args.path, "layout": args.layout, "us_median": out, "k_sweep": sweep}, indent=1))


def ctypes_int():
    import ctypes
    return ctypes.c_int


if __name__ == "__main__":
    main()
