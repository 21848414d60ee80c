"""Data parallelism for the Chebyshev path: one process per GPU, batch sharded,
L~ and W replicated, ONE all-reduce(sum) of the flat gradient bucket per step
inserted between compute_gradients and apply_gradients
(lib/graph_model.py:296-298).  Backend "nccl" is RCCL over xGMI on ROCm; "gloo"
is used for the CPU tests.  Gradient buckets on this path are a few KB
(SURVEY.md §8e), so the exchange is latency-bound: a single fused call.
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.distributed as dist

from . import _lib


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


def share_unique_id(uid: bytes, group=None, device=None) -> bytes:
    """Rank 0's 128-byte communicator id, broadcast to every rank of ``group``
    (the out-of-band step RCCL leaves to the caller).  nccl groups broadcast
    a device tensor, gloo groups a host tensor."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return bytes(uid)
    t = torch.frombuffer(bytearray(bytes(uid).ljust(128, b"\0")[:128]), dtype=torch.uint8).clone()
    if dist.get_backend(group) == "nccl":
        t = t.cuda(device)
    dist.broadcast(t, src=0, group=group)
    return bytes(t.cpu().tolist())


class TorchComm:
    """The gradient exchange of a training step (``allreduce_sum_`` + ``world``,
    the interface ResGNN / bench use) over a torch.distributed process group:
    a ProcessGroupNCCL (RCCL) all_reduce on the device tensor, or -- for gloo
    groups, e.g. ranks that share one GPU in a test -- through a host copy."""

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.backend = dist.get_backend(group) if dist.is_initialized() else None

    def allreduce_sum_(self, t: torch.Tensor, stream=None):
        """In-place SUM over ranks (enqueued after the work on t's current
        stream; ``stream`` is accepted for interface parity and must be that stream)."""
        if self.world == 1:
            return t
        if self.backend == "nccl" or not t.is_cuda:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        else:
            host = t.detach().cpu()
            dist.all_reduce(host, op=dist.ReduceOp.SUM, group=self.group)
            t.copy_(host)
        return t

    def close(self):
        pass


class RcclComm:
    """An RCCL communicator of libcheb_mi355 (cg_comm_* in the C ABI) over the
    ranks of a torch.distributed group: rank 0 creates the unique id, the group
    broadcasts it, every rank joins.  ``allreduce_sum_`` enqueues ncclAllReduce
    directly on the caller's HIP stream -- no side stream and no event
    fork/join around it (what ProcessGroupNCCL adds to every collective), so a
    step's gradient exchange is one kernel in stream order.  With no process
    group (single process) it is a 1-rank communicator."""

    def __init__(self, device: int, group=None):
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        uid = ctypes.create_string_buffer(128)
        if self.rank == 0:
            _lib.call("cg_comm_unique_id", uid)
        if self.world > 1:
            uid = ctypes.create_string_buffer(share_unique_id(uid.raw, group, device), 128)
        h = ctypes.c_void_p()
        _lib.call("cg_comm_init", ctypes.byref(h), self.world, self.rank, uid, int(device))
        self._h = h
        self._fn = _lib.lib().cg_allreduce_sum_f32

    @property
    def handle(self):
        return self._h

    def allreduce_sum_(self, t: torch.Tensor, stream=None):
        """In-place SUM over ranks of a contiguous fp32 device tensor."""
        if not t.is_cuda or t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError("allreduce_sum_ needs a contiguous fp32 device tensor")
        s = stream if stream is not None else torch.cuda.current_stream(t.device).cuda_stream
        _lib.check("cg_allreduce_sum_f32", self._fn(self._h, t.data_ptr(), t.numel(), s))
        return t

    def nranks(self) -> int:
        """Ranks the RCCL communicator spans (cg_comm_count = ncclCommCount)."""
        n = ctypes.c_int(0)
        _lib.call("cg_comm_count", self._h, ctypes.byref(n))
        return n.value

    def async_error(self, abort: bool = False) -> int:
        """Poll the communicator's asynchronous error (cg_comm_async_error):
        0 when healthy, else the RCCL result code (with ``abort`` the
        communicator is aborted so blocked ranks return)."""
        st = ctypes.c_int(0)
        rc = _lib.lib().cg_comm_async_error(self._h, ctypes.byref(st), int(abort))
        if rc not in (_lib.CG_OK, _lib.CG_ERR_COMM):
            _lib.check("cg_comm_async_error", rc)
        return st.value

    def close(self):
        if self._h is not None and self._h.value:
            _lib.lib().cg_comm_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
