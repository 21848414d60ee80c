#!/usr/bin/env python3
"""A/B of the 16- vs 8-channel group kernels on config R's hidden-layer shape
(M = 1024 graph of config E, Fin = Fout = 32, K = 20): the basis and dx must be
bitwise equal, y within fp32 rounding.  Runs each variant in a child process
(CG_GRP16 is read once per process) and compares the saved tensors."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(out):
    import scipy.sparse
    import torch
    sys.path.insert(0, ROOT)
    from cnn_graph_amd import ops
    from cnn_graph_amd.plan import ChebPlan
    with np.load(os.path.join(ROOT, "tests", "golden", "golden_E.npz"), allow_pickle=False) as z:
        M = int(z["M"])
        Lt = scipy.sparse.csr_matrix((z["Lt_val"], z["Lt_col"], z["Lt_rowptr"]), shape=(M, M))
    dev = torch.device("cuda", 0)
    plan = ChebPlan(Lt, device=0)
    N, Fin, K, Fout = 6, 32, 20, 32
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    x = torch.rand((N, M, Fin), device=dev, generator=g)
    W = torch.randn((Fin * K, Fout), device=dev, generator=g) * 0.1
    dy = torch.randn((N, M, Fout), device=dev, generator=g)
    r = ops.ChebRunner(plan, N, Fin, K, Fout, dev, basis_layout="planes")
    y = r.forward(x, W)
    basis = r.basis.clone()
    dx, dW = r.backward(dy, W)
    torch.cuda.synchronize()
    np.savez(out, y=y.cpu().numpy(), dx=dx.cpu().numpy(), dW=dW.cpu().numpy(),
             basis=basis.cpu().numpy())


def main():
    if len(sys.argv) > 1:
        child(sys.argv[1])
        return
    res = {}
    for v in ("1", "0"):
        out = f"/tmp/grp16_{v}.npz"
        env = dict(os.environ, CG_GRP16=v)
        subprocess.run([sys.executable, os.path.abspath(__file__), out], env=env, check=True)
        res[v] = dict(np.load(out))
    for k in res["1"]:
        a, b = res["1"][k], res["0"][k]
        d = float(np.abs(a.astype(np.float64) - b).max() / max(np.abs(b).max(), 1e-30))
        print(k, "bitwise" if np.array_equal(a, b) else f"normwise {d:.3e}")


if __name__ == "__main__":
    main()
