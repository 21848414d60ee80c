"""World-size-2 data-parallel logic on CPU (gloo): batch sharding + ONE fused
gradient all-reduce reproduces the full-batch gradient and keeps replicas in
lock-step.  Per-shard gradients come from the oracle (test infrastructure
standing in for the device kernels, which need a GPU).  Also the exchange
objects the training step drives (dist.TorchComm.allreduce_sum_ on a flat
buffer laid out like ResGNN's, and the RCCL unique-id broadcast of
dist.RcclComm, share_unique_id) over a real 2-rank gloo group.  The same step
with the HIP kernels at world size 2 is tests/test_gpu_dp.py."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, case, load_golden


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from cnn_graph_amd import dist as cdist
    from oracle import cheb_oracle as O
    try:
        r, w, _ = cdist.init(backend="gloo")
        assert (r, w) == (rank, world)
        c = case(load_golden("golden_A.npz"))
        N = c["N"]
        lo, hi = cdist.shard(N, rank, world)
        xs, dys = c["x"][lo:hi], c["dy"][lo:hi]
        basis, _ = O.cheb_forward(xs, c["Lt_rowptr"], c["Lt_col"], c["Lt_val"], c["W"], c["K"])
        _, dW = O.cheb_backward(dys, basis, c["W"], c["Lt_rowptr"], c["Lt_col"], c["Lt_val"],
                                hi - lo, c["M"], c["Fin"], c["K"])
        g1 = torch.tensor(dW, dtype=torch.float64)
        g2 = torch.full((3, 2), float(rank + 1), dtype=torch.float64)
        cdist.allreduce_gradients([g1, g2], average=False)
        W = torch.tensor(c["W"]) * (rank + 1)
        cdist.broadcast_parameters([W])
        # the exchange object of ResGNN.train_step on a flat gradient buffer
        # whose views are the per-layer gradients (one collective per step)
        flat = torch.arange(12, dtype=torch.float32) * (rank + 1)
        views = [flat[:5].view(5, 1), flat[5:].view(7, 1)]
        comm = cdist.TorchComm()
        assert comm.world == world and comm.rank == rank
        comm.allreduce_sum_(flat)
        assert torch.equal(views[1].flatten(), torch.arange(5, 12, dtype=torch.float32) * 3)
        # RcclComm's out-of-band unique-id step: rank 0's bytes everywhere
        uid = bytes([rank * 7 + i % 5 for i in range(128)])
        got = cdist.share_unique_id(uid)
        assert got == bytes([i % 5 for i in range(128)]), "unique id not rank 0's"
        q.put((rank, g1.numpy(), g2.numpy(), W.numpy()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surface the error to the parent
        q.put((rank, repr(e), None, None))


@pytest.mark.timeout(300)
def test_dp_world2_matches_full_batch():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, g1, g2, W = q.get(timeout=240)
        assert not isinstance(g1, str), g1
        res[rank] = (g1, g2, W)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from oracle import cheb_oracle as O
    c = case(load_golden("golden_A.npz"))
    basis, _ = O.cheb_forward(c["x"], c["Lt_rowptr"], c["Lt_col"], c["Lt_val"], c["W"], c["K"])
    _, dW_full = O.cheb_backward(c["dy"], basis, c["W"], c["Lt_rowptr"], c["Lt_col"], c["Lt_val"],
                                 c["N"], c["M"], c["Fin"], c["K"])
    for r in range(world):
        g1, g2, W = res[r]
        np.testing.assert_allclose(g1, dW_full, rtol=1e-12, atol=1e-12)
        np.testing.assert_array_equal(g2, np.full((3, 2), 3.0))
        np.testing.assert_array_equal(W, c["W"])        # rank 0's weights everywhere
    np.testing.assert_array_equal(res[0][0], res[1][0])  # replicas bitwise in sync


def test_shard_covers_batch():
    from cnn_graph_amd.dist import shard
    for n, w in ((256, 8), (10, 3), (7, 7)):
        spans = [shard(n, r, w) for r in range(w)]
        assert spans[0][0] == 0 and spans[-1][1] == n
        assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
