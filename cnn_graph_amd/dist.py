"""Data parallelism for the Chebyshev path: one process per GPU, batch sharded,
L~ and W replicated, ONE all-reduce(sum) of the flat gradient bucket per step
inserted between compute_gradients and apply_gradients
(lib/graph_model.py:296-298).  Backend "nccl" is RCCL over xGMI on ROCm; "gloo"
is used for the CPU tests.  Gradient buckets on this path are a few KB
(SURVEY.md §8e), so the exchange is latency-bound: a single fused call.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def env_rank_world():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), \
        int(os.environ.get("LOCAL_RANK", "0"))


def init(backend: str | None = None):
    """Initialise the default process group from the torchrun environment."""
    rank, world, local = env_rank_world()
    if world <= 1 or dist.is_initialized():
        return rank, world, local
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group(backend, rank=rank, world_size=world,
                                device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)
    return rank, world, local


def allreduce_gradients(grads, average=True, group=None):
    """Sum (or average) a list of gradient tensors across ranks in ONE
    collective over a flat bucket; returns the list (updated in place)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1 or not grads:
        return grads
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    if average:
        flat.div_(dist.get_world_size(group))
    off = 0
    for g in grads:
        n = g.numel()
        g.copy_(flat[off:off + n].view_as(g))
        off += n
    return grads


def broadcast_parameters(params, src=0, group=None):
    """Make every replica start from rank src's weights."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    for p in params:
        dist.broadcast(p.data, src=src, group=group)


def shard(n_global: int, rank: int, world: int):
    """Contiguous batch shard [lo, hi) of rank (last shard takes the remainder)."""
    per = n_global // world
    lo = rank * per
    hi = n_global if rank == world - 1 else lo + per
    return lo, hi
