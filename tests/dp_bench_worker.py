"""Worker of tests/test_gpu_dp_bench.py (not a test module): one rank of
bench.py's data-parallel step schedule (cnn_graph_amd/dp_step.py: forward-
applied Adam with W / m / v double-buffered, the dW all-reduce between
backward and the next forward, grad_scale = 1/world) on config B's graph,
launched by ``torch.distributed.run --nproc-per-node 2``.  Both ranks share
cuda:0 and exchange over gloo (dist.TorchComm; RCCL refuses two ranks on one
GPU).  Rank r runs its contiguous shard of a fixed global batch; rank 0 writes
both replicas' weights after every step for the parent to compare.

  python -m torch.distributed.run --nproc-per-node 2 tests/dp_bench_worker.py OUT.npz
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

STEPS = 3
N_GLOBAL, K, FOUT = 32, 25, 32


def problem():
    """Config B's graph (the reference MNIST recipe, M = 976), x with fake
    vertices 0, a fixed upstream dy and the initial W, shared by every rank."""
    import scipy.sparse
    from conftest import load_golden
    g = load_golden("golden_B.npz")
    L = scipy.sparse.csr_matrix((g["L_data"], g["L_indices"], g["L_indptr"]), shape=tuple(g["L_shape"]))
    M = L.shape[0]
    rng = np.random.default_rng(2017)
    x = rng.random((N_GLOBAL, M, 1), dtype=np.float32)
    x[:, g["fake_rows"], :] = 0
    dy = rng.standard_normal((N_GLOBAL, M, FOUT)).astype(np.float32)
    W0 = (rng.standard_normal((K, FOUT)) * 0.1).astype(np.float32)
    return L, x, dy, W0


def run(x, dy, W0, L, dev, world, allreduce_with, schedule, layout="orders", grad_scale=None):
    """STEPS steps of the schedule; returns the weights after each step [STEPS, K, Fout]."""
    import torch
    from cnn_graph_amd import ops
    from cnn_graph_amd.dp_step import ChebTrainStep
    from cnn_graph_amd.plan import ChebPlan
    plan = ChebPlan.from_laplacian(L, lmax=2, device=dev.index or 0)
    N = x.shape[0]
    runner = ops.ChebRunner(plan, N, 1, K, FOUT, dev, basis_layout=layout)
    tt = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    xs, dys = tt(x), tt(dy)
    allreduce = None if allreduce_with is None else (lambda s: allreduce_with(runner.dW, s))
    out = []
    for n in range(1, STEPS + 1):  # n steps from the same start, then the pending update
        tr = ChebTrainStep(runner, xs, dys, tt(W0), world=world, allreduce=allreduce,
                           schedule=schedule, grad_scale=grad_scale)
        s = torch.cuda.current_stream(dev).cuda_stream
        for i in range(n):
            tr.step(i, s)
        out.append(tr.finish(n, s).cpu().numpy().copy())
    torch.cuda.synchronize()
    return np.stack(out)


def main():
    import torch
    import torch.distributed as dist
    from cnn_graph_amd import dist as cdist
    out = sys.argv[1]
    rank, world, _ = cdist.init(backend="gloo")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    L, x, dy, W0 = problem()
    lo, hi = cdist.shard(N_GLOBAL, rank, world)
    comm = cdist.TorchComm()
    Ws = run(x[lo:hi], dy[lo:hi], W0, L, dev, world, lambda t, s: comm.allreduce_sum_(t, s),
             "forward")
    gathered = [torch.zeros(Ws.size, dtype=torch.float32) for _ in range(world)]
    dist.all_gather(gathered, torch.from_numpy(Ws.reshape(-1)))
    if rank == 0:
        np.savez(out, W=Ws, W_r1=gathered[1].numpy().reshape(Ws.shape), world=world)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
