"""Worker of tests/test_gpu_dp.py (not a test module): one rank of a
data-parallel ResGNN training step on the HIP kernels, launched by
``torch.distributed.run --nproc-per-node 2``.  Both ranks share cuda:0 and
exchange through a gloo group (dist.TorchComm; RCCL refuses two ranks on one
GPU), which is the same ResGNN.train_step code path the RCCL comm drives at
N > 1.  Rank r trains on its contiguous shard of a fixed global batch and
rank 0 writes what the parent compares with a one-process full-batch run.

  python -m torch.distributed.run --nproc-per-node 2 tests/dp_resgnn_worker.py OUT.npz
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

STEPS = 3
N_GLOBAL, FIN, NFILTER, K, NRES = 8, 2, 8, 4, 1


def problem():
    """Graph (golden A's Laplacian), inputs and labels shared by every rank."""
    import scipy.sparse
    from conftest import load_golden
    g = load_golden("golden_A.npz")
    L = scipy.sparse.csr_matrix((g["L_data"], g["L_indices"], g["L_indptr"]), shape=tuple(g["L_shape"]))
    M = L.shape[0]
    rng = np.random.default_rng(7)
    x = rng.standard_normal((N_GLOBAL, M, FIN)).astype(np.float32)
    labels = rng.standard_normal((N_GLOBAL, M, 2)).astype(np.float32)
    return L, x, labels


def run(N, x, labels, L, comm, dev):
    """STEPS train steps; returns (losses, grad after step 1, flat params)."""
    import torch
    from cnn_graph_amd.model import ResGNN
    net = ResGNN(L, N, FIN, NFILTER, K, NRES, device=dev, comm=comm, seed=2017)
    xt = torch.from_numpy(x).to(dev)
    lt = torch.from_numpy(labels).to(dev)
    losses, g1 = [], None
    for s in range(STEPS):
        losses.append(float(net.train_step(xt, lt).item()))
        if s == 0:
            g1 = net.grad.detach().cpu().numpy().copy()
    torch.cuda.synchronize()
    return np.array(losses), g1, net.flat.detach().cpu().numpy()


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
    losses, g1, flat = run(hi - lo, x[lo:hi], labels[lo:hi], L, comm, dev)
    loss_t = torch.tensor(losses, dtype=torch.float64)
    dist.all_reduce(loss_t)          # mean of the shard means = full-batch mean
    flats = [torch.zeros(flat.size, dtype=torch.float32) for _ in range(world)]
    dist.all_gather(flats, torch.from_numpy(flat))
    if rank == 0:
        np.savez(out, loss=loss_t.numpy() / world, grad1=g1 / world, flat=flat,
                 flat_r1=flats[1].numpy(), world=world)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
