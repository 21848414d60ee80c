"""A/B helper for k_lstm_seq variants (scratch): config E's layer forward and
fwd+bwd with a seeded cell; dumps hs and the parameter gradients to OUT.npz
(for a bitwise comparison between two library builds, chosen by CG_LIB_PATH)
and prints the event-timed forward / fwd+bwd.
    CG_LIB_PATH=... python scripts/ab_seq.py OUT [--cmp OTHER.npz]"""
import argparse
import json
import os
import sys

import numpy as np
import scipy.sparse
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--cmp", default=None)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from cnn_graph_amd.gconv_lstm import GConvLSTMCell, layer
    dev = torch.device("cuda", 0)
    with np.load(os.path.join(ROOT, "tests", "golden", "golden_E.npz"), allow_pickle=False) as z:
        M = int(z["M"])
        Lt = scipy.sparse.csr_matrix((z["Lt_val"], z["Lt_col"], z["Lt_rowptr"]), shape=(M, M))
    L = (Lt + scipy.sparse.identity(M, dtype=np.float32, format="csr")).tocsr()
    T, N, Fin, H, K = 12, 128, 2, 32, 3
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    cell = GConvLSTMCell(H, laplacian=L, lmax=2, K=K, feat_in=Fin, device=dev, generator=g)
    xs = torch.rand((T, N, M, Fin), device=dev, generator=g)
    gh = torch.randn((T, N, M, H), device=dev, generator=g)
    hs, _ = layer(cell, xs)
    hs.backward(gh)
    torch.cuda.synchronize()
    res = {"hs": hs.detach().cpu().numpy()}
    for i, p in enumerate(cell.parameters()):
        res[f"g{i}"] = p.grad.cpu().numpy()
    np.savez(a.out, **res)
    if a.cmp:
        with np.load(a.cmp, allow_pickle=False) as z:
            same = {k: bool(np.array_equal(z[k], res[k])) for k in res}
        print(json.dumps({"bitwise": same}))
        if not all(same.values()):
            sys.exit(3)

    def fwd():
        with torch.no_grad():
            layer(cell, xs)

    def fwdbwd():
        for p in cell.parameters():
            p.grad = None
        h, _ = layer(cell, xs)
        h.backward(gh)

    out = {}
    for name, fn in (("fwd_ms", fwd), ("fwd_bwd_ms", fwdbwd)):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        out[name] = round(float(np.median(ts)), 4)
    out["lib"] = os.path.basename(os.environ.get("CG_LIB_PATH", "libcheb_mi355.so"))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
