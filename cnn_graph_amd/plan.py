"""Device plan of one rescaled Laplacian: the analogue of the TF graph constant
that ``chebyshev5`` builds from ``L`` at lib/graph_conv.py:148-153.

A plan owns device copies of L~ (CSR) and L~^T and is cached per (L object,
lmax, device), since the reference's eager callers pass the same scipy matrix
to every filter call (lib/graph_conv.py:241, 246, 312, 324 all use L[0]).
Like TF's constant folding, the cache snapshots L at first use: do not mutate
L in place afterwards (call ``clear_plan_cache()`` if you must).
"""
from __future__ import annotations

import ctypes
import weakref

import numpy as np

from . import _lib
from . import graph as _graph


def _i32p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


def _f32p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


class ChebPlan:
    """Owns a ``cg_plan`` (device CSR of L~ and L~^T)."""

    def __init__(self, Lt, device: int = 0, path: str = "auto", variant: str = "auto"):
        rowptr, col, val = _graph.canonical_csr(Lt)
        self.M = int(Lt.shape[0])
        self.nnz = int(len(col))
        self.device = int(device)
        self.rowptr, self.col, self.val = rowptr, col, val
        h = ctypes.c_void_p()
        _lib.call("cg_plan_create", ctypes.byref(h), self.device, self.M, self.nnz,
                  _i32p(rowptr), _i32p(col), _f32p(val), None, None, None)
        self._h = h
        self._lib = _lib.lib()
        self._ws = {}
        self.set_variant(variant)
        self.set_path(path)

    @classmethod
    def from_laplacian(cls, L, lmax=2, device: int = 0, path: str = "auto", variant: str = "auto"):
        """L~ = rescale_L(L, lmax) then a plan (lib/graph_conv.py:148-149)."""
        return cls(_graph.rescale_L(L, lmax), device=device, path=path, variant=variant)

    @property
    def handle(self):
        return self._h

    def set_path(self, path: str):
        _lib.call("cg_plan_set_path", self._h, _lib.PATHS[path])
        self.path = path
        self._shape_cache = {}

    def set_variant(self, variant: str):
        """Kernel variant ('auto', 'classic', 'unfused_dw'): same results, other kernels."""
        _lib.call("cg_plan_set_variant", self._h, _lib.VARIANTS[variant])
        self.variant = variant
        self._shape_cache = {}

    def set_seq_fault_test(self, step: int):
        """Failure-detection test hook (cg_plan_set_seq_fault_test): from time step
        ``step`` on, this plan's gconv-LSTM sequence launches lose one pair
        hand-off; -1 turns it off."""
        _lib.call("cg_plan_set_seq_fault_test", self._h, int(step))

    # workspaces above this size are not kept by the plan (a config-D backward
    # at N = 256 needs 51.5 GB: holding it for the plan's lifetime would pin it
    # for every later model that shares the plan through plan_for)
    WS_CACHE_MAX_BYTES = 1 << 30

    def workspace(self, nbytes: int, device, stream_id: int):
        """A device workspace of at least ``nbytes``.  Up to WS_CACHE_MAX_BYTES
        it is owned by the plan and reused by every call enqueued on the same
        stream (stream order makes the reuse safe: a call's workspace is dead
        once the call has executed); grown, never shrunk, one buffer per
        (device, stream) -- ``release_workspace()`` frees them.  Larger requests
        get a buffer of their own that the caching allocator takes back once the
        call's stream has used it (torch's stream-ordered frees)."""
        import torch
        nbytes = max(int(nbytes), 256)
        if nbytes > self.WS_CACHE_MAX_BYTES:
            return torch.empty(nbytes, device=device, dtype=torch.uint8)
        key = (str(device), int(stream_id))
        buf = self._ws.get(key)
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(nbytes, device=device, dtype=torch.uint8)
            self._ws[key] = buf
        return buf

    def release_workspace(self):
        """Drop the plan's cached workspaces (e.g. after a large streaming call,
        or when the stream they were keyed on is gone)."""
        self._ws = {}

    def _shape_info(self, N, Fin, K, Fout):
        key = (int(N), int(Fin), int(K), int(Fout))
        info = self._shape_cache.get(key)
        if info is None:
            out = ctypes.c_int()
            _lib.call("cg_plan_query_path", self._h, *key, ctypes.byref(out))
            f, b = ctypes.c_size_t(), ctypes.c_size_t()
            _lib.call("cg_cheb_workspace_bytes", self._h, *key, ctypes.byref(f), ctypes.byref(b))
            path = {v: k for k, v in _lib.PATHS.items()}[out.value]
            info = (path, int(f.value), int(b.value))
            self._shape_cache[key] = info
        return info

    def query_path(self, N, Fin, K, Fout) -> str:
        """'resident' or 'stream': the kernel path the forward takes for this shape."""
        return self._shape_info(N, Fin, K, Fout)[0]

    def workspace_bytes(self, N, Fin, K, Fout):
        """(forward, backward) device workspace bytes for this shape."""
        return self._shape_info(N, Fin, K, Fout)[1:]

    def basis_elems(self, N, Fin, K, Fout, layout: str = "rows"):
        """Floats of the basis buffer in ``layout`` ('rows' [N*M, Fin*K], 'orders'
        [N, Fin*K, Mb] or 'planes' [K, N*M, Fin]), or None where the layout does
        not apply to this shape (cg_cheb_basis_elems)."""
        n = ctypes.c_int64()
        st = self._lib.cg_cheb_basis_elems(self._h, N, Fin, K, Fout, _lib.BASIS_LAYOUTS[layout],
                                           ctypes.byref(n))
        if st == 3:  # CG_ERR_UNSUPPORTED
            return None
        _lib.check("cg_cheb_basis_elems", st)
        return int(n.value)

    def close(self):
        self._ws = {}
        if getattr(self, "_h", None) is not None and self._h.value:
            self._lib.cg_plan_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_CACHE: dict = {}


def _evict(key):
    plan = _CACHE.pop(key, None)
    if plan is not None:
        plan[0].close()


def plan_for(L, lmax=2, device: int = 0, path: str = "auto") -> ChebPlan:
    """Cached plan for the scipy Laplacian ``L`` (rescaled with ``lmax``)."""
    key = (id(L), float(lmax), int(device))
    hit = _CACHE.get(key)
    if hit is not None:
        plan, shape, nnz = hit
        if shape == L.shape and nnz == L.nnz:
            if plan.path != path:
                plan.set_path(path)
            return plan
        _evict(key)
    plan = ChebPlan.from_laplacian(L, lmax=lmax, device=device, path=path)
    _CACHE[key] = (plan, L.shape, L.nnz)
    try:
        weakref.finalize(L, _evict, key)
    except TypeError:
        pass
    return plan


def clear_plan_cache():
    for key in list(_CACHE):
        _evict(key)
