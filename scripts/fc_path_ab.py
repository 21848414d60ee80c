"""Config E's model step with the fc layer's chebyshev5 on other kernel
paths / variants of the same plan (the LSTM kernels do not consult either):
ms per train step, and the loss after the steps (same seeds)."""
import json
import os
import sys

import numpy as np
import scipy.sparse
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from cnn_graph_amd.gconv_lstm import GLSTMModel
    dev = torch.device("cuda", 0)
    T, Fin, H, K, Fout, N = 12, 2, 32, 3, 2, 128
    with np.load(os.path.join(ROOT, "tests", "golden", "golden_E.npz"), allow_pickle=False) as z:
        M = int(z["M"])
        Lt = scipy.sparse.csr_matrix((z["Lt_val"], z["Lt_col"], z["Lt_rowptr"]), shape=(M, M))
    L = (Lt + scipy.sparse.identity(M, dtype=np.float32, format="csr")).tocsr()
    g = torch.Generator(device=dev)
    g.manual_seed(2017)
    x = torch.rand((N, M, Fin * T), device=dev, generator=g)
    labels = torch.rand((N, M, Fout), device=dev, generator=g)
    for setting in sys.argv[1:] or ["auto", "steps", "stream", "auto"]:
        model = GLSTMModel(L, N, T, Fin, num_hidden=H, K=K, out_features=Fout, keep_prob=0.8,
                           device=dev, seed=2017)
        if setting == "stream":
            model.plan.set_path("stream")
        elif setting != "auto":
            model.plan.set_variant(setting)
        s = torch.cuda.current_stream(dev).cuda_stream
        for _ in range(3):
            model.train_step(x, labels, s)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(30):
            model.train_step(x, labels, s)
        e1.record()
        torch.cuda.synchronize()
        print(json.dumps({"setting": setting, "ms_per_step": round(e0.elapsed_time(e1) / 30, 4),
                          "loss": float(model.loss.item()),
                          "path": model.plan.query_path(N, H, K, Fout)}), flush=True)
        model.plan.set_path("auto")
        model.plan.set_variant("auto")


if __name__ == "__main__":
    main()
