#!/usr/bin/env python3
"""A/B of the gconv-LSTM sequence forward with the x basis precomputed for all
steps (CG_SEQ_XPRE=1, default) vs recomputed inside the loop (0), config E's
shape (M = 1024, T = 12, N = 128, Fin = 2, H = 32, K = 3): hs, cs, act and the
x planes must be bitwise equal.  Each mode runs in a child process (the switch
is read once per process)."""
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
    T, N, H, K, Fin = 12, 128, 32, 3, 2
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    Wh = torch.randn((K * H, 4 * H), device=dev, generator=g) * 0.1
    b = torch.randn((4 * H,), device=dev, generator=g) * 0.1
    xs = torch.rand((T, N, M, Fin), device=dev, generator=g)
    Wx = torch.randn((K * Fin, 4 * H), device=dev, generator=g) * 0.1
    hs = torch.empty((T, N, M, H), device=dev)
    cs = torch.empty_like(hs)
    act = torch.empty((T, N, M, 4 * H), device=dev)
    planes = torch.empty((K - 1, T, N * M, H), device=dev)
    xpl = torch.empty((K, T * N * M, Fin), device=dev)
    ops.lstm_seq_forward_x(plan, xs, Wx, Wh, b, K, out_hs=hs, out_cs=cs, out_act=act,
                           planes=planes[0], plane_stride=T * N * M * H, xplanes=xpl)
    torch.cuda.synchronize()
    np.savez(out, hs=hs.cpu().numpy(), cs=cs.cpu().numpy(), act=act.cpu().numpy(),
             planes=planes.cpu().numpy(), xpl=xpl.cpu().numpy())


def main():
    if len(sys.argv) > 1:
        child(sys.argv[1])
        return
    res = {}
    for v in ("1", "0"):
        out = f"/tmp/seqxpre_{v}.npz"
        subprocess.run([sys.executable, os.path.abspath(__file__), out],
                       env=dict(os.environ, CG_SEQ_XPRE=v), check=True)
        res[v] = dict(np.load(out))
    for k in res["1"]:
        a, b = res["1"][k], res["0"][k]
        d = float(np.abs(a.astype(np.float64) - b).max() / max(np.abs(b).max(), 1e-30))
        print(k, "bitwise" if np.array_equal(a, b) else f"normwise {d:.3e}")


if __name__ == "__main__":
    main()
