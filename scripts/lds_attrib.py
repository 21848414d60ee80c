#!/usr/bin/env python3
"""One config-B forward (cheb_fwd_fast, N = 256, the bench's orders layout) x 20
launches on the DEBUG build with ablation flags, for LDS bank-conflict
attribution under rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE (one
process per flag set, scripts/gpu_r04_lds.sh).  Forward flag bits: 2 no basis
kept, 4 no MFMA, 8 no y store, 16 prologue only, 64 no gathers, 128 no
own-record writes (outputs are garbage when set; counters only).
  python3 scripts/lds_attrib.py FLAGS"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("CG_LIB_PATH", os.path.join(ROOT, "scripts", "dbg", "libcheb_mi355_debug.so"))
import bench  # noqa: E402
from cnn_graph_amd import _lib, ops  # noqa: E402
from cnn_graph_amd.plan import ChebPlan  # noqa: E402


def main():
    flags = int(sys.argv[1])
    dev = torch.device("cuda", 0)
    L, _ = bench.load_config_b()
    K, Fin, Fout, N = 25, 1, 32, 256
    plan = ChebPlan.from_laplacian(L, 2, 0)
    x = torch.rand((N, plan.M, Fin), device=dev)
    W = torch.randn((K, Fout), device=dev) * 0.1
    r = ops.ChebRunner(plan, N, Fin, K, Fout, dev, basis_layout="orders")
    h = _lib.lib()
    h.cg_debug_set_flags.argtypes = [ctypes.c_int]
    h.cg_debug_set_flags(flags)
    for _ in range(20):
        r.forward(x, W)
    torch.cuda.synchronize()
    h.cg_debug_set_flags(0)
    print("ok", flags)


if __name__ == "__main__":
    main()
