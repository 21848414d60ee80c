"""PyTorch-facing ops over the HIP kernels (device memory, streams, autograd).

PyTorch is plumbing here: every op hands raw device pointers and the current
HIP stream to libcheb_mi355.so.  There is no CPU/eager fallback: a CPU tensor
or a missing library raises.

  cheb_forward / cheb_backward  -- lib/graph_conv.py:144-176 and its TF autodiff
  ChebConv (autograd.Function)  -- what chebyshev5 / cheby_conv call
  mpool1, apool1                -- lib/graph_conv.py:201-218
  perm_data                     -- lib/coarsening.py:219-240 (device gather)
  adam_update                   -- lib/graph_model.py:293-298
"""
from __future__ import annotations

import torch

from . import _lib
from .plan import ChebPlan


def _stream(t: torch.Tensor):
    return torch.cuda.current_stream(t.device).cuda_stream


def _check_dev(name, t: torch.Tensor, dtype=torch.float32):
    if not t.is_cuda:
        raise ValueError(f"{name}: expected a HIP (cuda) tensor, got {t.device}; "
                         "cnn_graph_amd has no CPU path")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")


def _p(t):
    return None if t is None else t.data_ptr()


def cheb_forward(plan: ChebPlan, x: torch.Tensor, W: torch.Tensor | None, K: int,
                 want_basis: bool = True):
    """Basis (N*M, Fin*K) and y = basis @ W (N, M, Fout).  W None -> basis only."""
    _check_dev("x", x)
    x = x.contiguous()
    N, M, Fin = x.shape
    if M != plan.M:
        raise ValueError(f"x has M={M} vertices but the Laplacian has {plan.M}")
    if W is not None:
        _check_dev("W", W)
        W = W.contiguous()
        if W.shape[0] != Fin * K:
            raise ValueError(f"W must be [Fin*K, Fout] = [{Fin * K}, *], got {tuple(W.shape)}")
        Fout = int(W.shape[1])
    else:
        Fout = 1
    dev = x.device
    # the streaming path's GEMM reads the basis from HBM, so it always needs one
    need_basis = want_basis or W is None or plan.query_path(N, Fin, K, Fout) == "stream"
    basis = torch.empty((N * M, Fin * K), device=dev, dtype=torch.float32) if need_basis else None
    y = torch.empty((N, M, Fout), device=dev, dtype=torch.float32) if W is not None else None
    fwd_ws, _ = plan.workspace_bytes(N, Fin, K, Fout)
    ws = torch.empty(max(fwd_ws, 1), device=dev, dtype=torch.uint8)
    _lib.call("cg_cheb_forward", plan.handle, N, Fin, K, Fout, _p(x), _p(W), _p(basis), _p(y),
              _p(ws), fwd_ws, _stream(x))
    return basis, y


def cheb_backward(plan: ChebPlan, dy: torch.Tensor, basis: torch.Tensor, W: torch.Tensor, K: int,
                  need_dx: bool = True):
    """(dx [N,M,Fin] or None, dW [Fin*K, Fout])."""
    _check_dev("dy", dy)
    dy = dy.contiguous()
    N, M, Fout = dy.shape
    FinK = int(W.shape[0])
    Fin = FinK // K
    dev = dy.device
    dx = torch.empty((N, M, Fin), device=dev, dtype=torch.float32) if need_dx else None
    dW = torch.empty((FinK, Fout), device=dev, dtype=torch.float32)
    _, bwd_ws = plan.workspace_bytes(N, Fin, K, Fout)
    ws = torch.empty(max(bwd_ws, 1), device=dev, dtype=torch.uint8)
    _lib.call("cg_cheb_backward", plan.handle, N, Fin, K, Fout, _p(dy), _p(basis), _p(W.contiguous()),
              _p(dx), _p(dW), _p(ws), bwd_ws, _stream(dy))
    return dx, dW


class ChebRunner:
    """Pre-allocated forward/backward of one (plan, N, Fin, K, Fout) shape:
    every device buffer (basis, y, dx, dW, workspaces) is allocated once, so a
    step is just the C-ABI launches on the current stream -- no allocator or
    Python-side shape work per call (and safe to capture in a HIP graph)."""

    def __init__(self, plan: ChebPlan, N: int, Fin: int, K: int, Fout: int, device):
        self.plan, self.N, self.Fin, self.K, self.Fout = plan, int(N), int(Fin), int(K), int(Fout)
        dev = torch.device(device)
        self.path = plan.query_path(N, Fin, K, Fout)
        fb, bb = plan.workspace_bytes(N, Fin, K, Fout)
        M = plan.M
        f32 = dict(device=dev, dtype=torch.float32)
        self.basis = torch.empty((N * M, Fin * K), **f32)
        self.y = torch.empty((N, M, Fout), **f32)
        self.dx = torch.empty((N, M, Fin), **f32)
        self.dW = torch.empty((Fin * K, Fout), **f32)
        self.fws = torch.empty(max(fb, 1), device=dev, dtype=torch.uint8)
        self.bws = torch.empty(max(bb, 1), device=dev, dtype=torch.uint8)
        self.fwd_bytes, self.bwd_bytes = fb, bb
        self._fwd = _lib.lib().cg_cheb_forward
        self._bwd = _lib.lib().cg_cheb_backward

    def forward(self, x: torch.Tensor, W: torch.Tensor, stream=None):
        s = stream if stream is not None else torch.cuda.current_stream(x.device).cuda_stream
        st = self._fwd(self.plan.handle, self.N, self.Fin, self.K, self.Fout, x.data_ptr(),
                       W.data_ptr(), self.basis.data_ptr(), self.y.data_ptr(), self.fws.data_ptr(),
                       self.fwd_bytes, s)
        _lib.check("cg_cheb_forward", st)
        return self.y

    def backward(self, dy: torch.Tensor, W: torch.Tensor, need_dx: bool = True, stream=None):
        s = stream if stream is not None else torch.cuda.current_stream(dy.device).cuda_stream
        st = self._bwd(self.plan.handle, self.N, self.Fin, self.K, self.Fout, dy.data_ptr(),
                       self.basis.data_ptr(), W.data_ptr(),
                       self.dx.data_ptr() if need_dx else None, self.dW.data_ptr(),
                       self.bws.data_ptr(), self.bwd_bytes, s)
        _lib.check("cg_cheb_backward", st)
        return (self.dx if need_dx else None), self.dW


class ChebConv(torch.autograd.Function):
    """y = chebyshev5(x; L~, W, K) with the HIP forward/backward kernels."""

    @staticmethod
    def forward(ctx, x, W, plan: ChebPlan, K: int):
        basis, y = cheb_forward(plan, x, W, K, want_basis=True)
        ctx.save_for_backward(basis, W)
        ctx.plan, ctx.K = plan, K
        return y

    @staticmethod
    def backward(ctx, dy):
        basis, W = ctx.saved_tensors
        dx, dW = cheb_backward(ctx.plan, dy, basis, W, ctx.K, need_dx=ctx.needs_input_grad[0])
        return dx, dW, None, None


def cheb_conv(x, W, plan: ChebPlan, K: int):
    return ChebConv.apply(x, W, plan, K)


class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p: int):
        _check_dev("x", x)
        x = x.contiguous()
        N, M, F = x.shape
        y = torch.empty((N, M // p, F), device=x.device, dtype=torch.float32)
        arg = torch.empty((N, M // p, F), device=x.device, dtype=torch.int32)
        _lib.call("cg_maxpool_forward", _p(x), N, M, F, p, _p(y), _p(arg), _stream(x))
        ctx.save_for_backward(arg)
        ctx.shape, ctx.p = (N, M, F), p
        ctx.mark_non_differentiable(arg)
        return y, arg

    @staticmethod
    def backward(ctx, dy, _darg):
        (arg,) = ctx.saved_tensors
        N, M, F = ctx.shape
        dy = dy.contiguous()
        dx = torch.empty((N, M, F), device=dy.device, dtype=torch.float32)
        _lib.call("cg_maxpool_backward", _p(dy), _p(arg), N, M, F, ctx.p, _p(dx), _stream(dy))
        return dx, None


def mpool1_with_argmax(x, p: int):
    """(y, argmax) -- argmax is the absolute vertex of the first maximum."""
    return _MaxPool.apply(x, p)


def mpool1(x, p: int):
    """Max pooling of size p along vertices (lib/graph_conv.py:201-209)."""
    if p <= 1:
        return x
    return _MaxPool.apply(x, p)[0]


class _AvgPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p: int):
        _check_dev("x", x)
        x = x.contiguous()
        N, M, F = x.shape
        y = torch.empty((N, M // p, F), device=x.device, dtype=torch.float32)
        _lib.call("cg_avgpool_forward", _p(x), N, M, F, p, _p(y), _stream(x))
        ctx.shape, ctx.p = (N, M, F), p
        return y

    @staticmethod
    def backward(ctx, dy):
        N, M, F = ctx.shape
        dy = dy.contiguous()
        dx = torch.empty((N, M, F), device=dy.device, dtype=torch.float32)
        _lib.call("cg_avgpool_backward", _p(dy), N, M, F, ctx.p, _p(dx), _stream(dy))
        return dx, None


def apool1(x, p: int):
    """Average pooling of size p along vertices (lib/graph_conv.py:211-218)."""
    if p <= 1:
        return x
    return _AvgPool.apply(x, p)


def perm_data(x: torch.Tensor, perm) -> torch.Tensor:
    """Device perm_data (lib/coarsening.py:219-240): x [N, M] or [N, M, F] ->
    [N, len(perm)(, F)] with fake vertices (perm[i] >= M) set to 0."""
    _check_dev("x", x)
    squeeze = x.dim() == 2
    x3 = (x.unsqueeze(-1) if squeeze else x).contiguous()
    N, M, F = x3.shape
    perm_t = torch.as_tensor(perm, dtype=torch.int32, device=x.device).contiguous()
    Mo = int(perm_t.numel())
    out = torch.empty((N, Mo, F), device=x.device, dtype=torch.float32)
    _lib.call("cg_perm_gather", _p(x3), _p(perm_t), N, M, Mo, F, _p(out), _stream(x))
    return out[..., 0] if squeeze else out


def adam_update(param, grad, m, v, step: int, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8,
                grad_scale=1.0):
    """In-place TF-1.x Adam step on device (lib/graph_model.py:293)."""
    for name, t in (("param", param), ("grad", grad), ("m", m), ("v", v)):
        _check_dev(name, t)
        if not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")
    _lib.call("cg_adam_update", _p(param), _p(grad), _p(m), _p(v), param.numel(), float(lr),
              float(beta1), float(beta2), float(eps), int(step), float(grad_scale), _stream(param))
