#!/usr/bin/env python3
"""Backward of config R's hidden-layer filter (M = 1024 graph of config E,
N = 100, Fin = Fout = 32, K = 20, planes layout) repeated 30 times, for kernel
traces under CG_CLEN_DY=0 (row GEMM dBasis planes + k_grp_clen), 1 (k_grp_clen_dy,
next group's tiles during the current group's steps), 2 (k_grp_clen_dy, each
group's tiles up front).  Prints the HIP-event time per backward call."""
import os
import sys

import numpy as np
import scipy.sparse
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cnn_graph_amd import ops  # noqa: E402
from cnn_graph_amd.plan import ChebPlan  # noqa: E402


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
    r.forward(x, W)
    for _ in range(5):
        r.backward(dy, W)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(30):
        r.backward(dy, W)
    e1.record()
    torch.cuda.synchronize()
    print(f"CG_CLEN_DY={os.environ.get('CG_CLEN_DY', '1')} backward {e0.elapsed_time(e1) / 30 * 1e3:.1f} us")


if __name__ == "__main__":
    main()
