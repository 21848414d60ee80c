"""Worker of tests/test_gpu_glstm_dp.py (not a test module): one rank of the
data-parallel gconv-LSTM training step (gconv_lstm.GLSTMModel: glstm_layer +
fc_layer + MSE + Adam, ONE all-reduce of the flat gradient bucket per step,
grad_scale = 1/world) at config E's graph and shape (T = 12, K = 3, H = 32,
Fin = 2), launched by ``torch.distributed.run --nproc-per-node 2``.  Both ranks
share cuda:0 and exchange over gloo (dist.TorchComm; RCCL refuses two ranks on
one GPU).  Rank r trains on its contiguous shard of a fixed global batch; rank
0 writes both replicas' parameters after every step and the first step's
exchanged gradient bucket for the parent to compare.

  python -m torch.distributed.run --nproc-per-node 2 tests/glstm_dp_worker.py OUT.npz
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

STEPS = 3
N_GLOBAL, T, FIN, H, K, FOUT = 8, 12, 2, 32, 3, 2


def problem():
    """Config E's graph (golden_E.npz: L~ of the 1024-vertex grid; the model is
    built from L = L~ + I so that rescale_L(L, 2) = L~), the input sequence as
    the reference feeds it ([N, M, Fin*T]) and the labels."""
    import scipy.sparse
    from conftest import case, load_golden
    c = case(load_golden("golden_E.npz"))
    M = c["M"]
    Lt = scipy.sparse.csr_matrix((c["Lt_val"], c["Lt_col"], c["Lt_rowptr"]), shape=(M, M))
    L = (Lt + scipy.sparse.identity(M, dtype=np.float32, format="csr")).tocsr()
    rng = np.random.default_rng(512)
    x = rng.random((N_GLOBAL, M, FIN * T), dtype=np.float32)
    labels = rng.random((N_GLOBAL, M, FOUT), dtype=np.float32)
    return L, x, labels


def run(L, x, labels, dev, comm, optimizer="adam"):
    """STEPS training steps; returns (params after each step [STEPS, P], the
    gradient bucket of step 1 divided by the world size [P], losses)."""
    import torch
    from cnn_graph_amd.gconv_lstm import GLSTMModel
    N = x.shape[0]
    model = GLSTMModel(L, N, T, FIN, num_hidden=H, K=K, out_features=FOUT, keep_prob=1.0,
                       optimizer=optimizer, device=dev, seed=2017, comm=comm)
    xs = torch.from_numpy(np.ascontiguousarray(x)).to(dev)
    ys = torch.from_numpy(np.ascontiguousarray(labels)).to(dev)
    params, losses, g1 = [], [], None
    for i in range(STEPS):
        loss = model.train_step(xs, ys)
        if i == 0:
            g1 = (model.grad / model.world).cpu().numpy().copy()
        params.append(model.flat.cpu().numpy().copy())
        losses.append(float(loss.item()))
    torch.cuda.synchronize()
    return np.stack(params), g1, np.array(losses)


def main():
    import torch
    import torch.distributed as dist
    from cnn_graph_amd import dist as cdist
    out = sys.argv[1]
    rank, world, _ = cdist.init(backend="gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    L, x, labels = problem()
    lo, hi = cdist.shard(N_GLOBAL, rank, world)
    comm = cdist.TorchComm()
    P, g1, losses = run(L, x[lo:hi], labels[lo:hi], dev, comm)
    gathered = [torch.zeros(P.size, dtype=torch.float32) for _ in range(world)]
    dist.all_gather(gathered, torch.from_numpy(P.reshape(-1)))
    if rank == 0:
        np.savez(out, P=P, P_r1=gathered[1].numpy().reshape(P.shape), g1=g1, world=world)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
