#!/usr/bin/env python3
"""A/B of the fused-dBasis Clenshaw kernel (k_grp_clen_dy) vs the row GEMM + k_grp_clen pair on config R's hidden-layer shape
(M = 1024 graph of config E, Fin = Fout = 32, K = 20): the basis and dx must be
bitwise equal (dx, dW, basis, y: the forward is untouched).  Runs each variant in a child process
(CG_CLEN_DY is read once per process) and compares the saved tensors."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


SHAPE = (6, 32, 20, 32, 0)  # N, Fin, K, Fout, graph (0: config E's M = 1024, 1: config B's M = 976)


def child(out):
    import scipy.sparse
    import torch
    sys.path.insert(0, ROOT)
    from cnn_graph_amd import ops
    from cnn_graph_amd.plan import ChebPlan
    gname = "golden_B.npz" if SHAPE[4] == 1 else "golden_E.npz"
    with np.load(os.path.join(ROOT, "tests", "golden", gname), allow_pickle=False) as z:
        M = int(z["M"])
        Lt = scipy.sparse.csr_matrix((z["Lt_val"], z["Lt_col"], z["Lt_rowptr"]), shape=(M, M))
    dev = torch.device("cuda", 0)
    plan = ChebPlan(Lt, device=0, path="stream")
    N, Fin, K, Fout = SHAPE[:4]
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    x = torch.rand((N, M, Fin), device=dev, generator=g)
    W = torch.randn((Fin * K, Fout), device=dev, generator=g) * 0.1
    dy = torch.randn((N, M, Fout), device=dev, generator=g)
    r = ops.ChebRunner(plan, N, Fin, K, Fout, dev, basis_layout="planes" if Fin % 16 == 0 else "rows")
    y = r.forward(x, W)
    basis = r.basis.clone()
    dx, dW = r.backward(dy, W)
    torch.cuda.synchronize()
    np.savez(out, y=y.cpu().numpy(), dx=dx.cpu().numpy(), dW=dW.cpu().numpy(),
             basis=basis.cpu().numpy())


def main():
    global SHAPE
    if len(sys.argv) > 2:
        SHAPE = tuple(int(v) for v in sys.argv[2].split(","))
    if len(sys.argv) > 1 and sys.argv[1] != "--shape":
        child(sys.argv[1])
        return
    for shape in ((6, 32, 20, 32, 0), (5, 16, 7, 64, 0), (4, 8, 2, 32, 0), (3, 24, 5, 32, 1),
                  (4, 32, 20, 32, 1)):
        SHAPE = shape
        compare()


def compare():
    res = {}
    for v in ("1", "0"):
        out = f"/tmp/clendy_{v}.npz"
        env = dict(os.environ, CG_CLEN_DY=v)
        subprocess.run([sys.executable, os.path.abspath(__file__), out, ",".join(map(str, SHAPE))],
                       env=env, check=True)
        res[v] = dict(np.load(out))
    for k in res["1"]:
        a, b = res["1"][k], res["0"][k]
        d = float(np.abs(a.astype(np.float64) - b).max() / max(np.abs(b).max(), 1e-30))
        print(SHAPE, k, "bitwise" if np.array_equal(a, b) else f"normwise {d:.3e}")


if __name__ == "__main__":
    main()
