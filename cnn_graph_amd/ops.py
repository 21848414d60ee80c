"""PyTorch-facing ops over the HIP kernels (device memory, streams, autograd).

PyTorch is plumbing here: every op hands raw device pointers and the current
HIP stream to libcheb_mi355.so.  There is no CPU/eager fallback: a CPU tensor
or a missing library raises.

  cheb_forward / cheb_backward  -- lib/graph_conv.py:144-176 and its TF autodiff
  ChebConv (autograd.Function)  -- what chebyshev5 / cheby_conv call
  bias_act                      -- b1relu / b1tanh / b2relu, lib/graph_conv.py:178-199
  matmul                        -- tf.matmul of fc, lib/graph_conv.py:220-226 (MFMA GEMM)
  fourier_conv                  -- filter_in_fourier, lib/graph_conv.py:83-111
  mpool1, apool1                -- lib/graph_conv.py:201-218
  perm_data                     -- lib/coarsening.py:219-240 (device gather)
  adam_update                   -- lib/graph_model.py:293-298
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .plan import ChebPlan


def _stream(t: torch.Tensor):
    return torch.cuda.current_stream(t.device).cuda_stream


def _plan_ws(plan: ChebPlan, nbytes: int, t: torch.Tensor):
    """(workspace tensor, stream) for a call on t's current stream: the plan's
    cached per-stream buffer (no allocation per autograd call)."""
    s = _stream(t)
    return plan.workspace(nbytes, t.device, s), s


def _check_dev(name, t: torch.Tensor, dtype=torch.float32):
    if not t.is_cuda:
        raise ValueError(f"{name}: expected a HIP (cuda) tensor, got {t.device}; "
                         "cnn_graph_amd has no CPU path")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")


def _p(t):
    return None if t is None else t.data_ptr()


def _check_out(name, t, shape):
    """A caller-supplied output: fp32, on the GPU, contiguous, with prod(shape) elements."""
    _check_dev(name, t)
    n = 1
    for s in shape:
        n *= int(s)
    if not t.is_contiguous() or t.numel() != n:
        raise ValueError(f"{name}: need a contiguous tensor of {tuple(shape)} elements, "
                         f"got {tuple(t.shape)}")


ACTS = {"none": _lib.CG_ACT_NONE, "relu": _lib.CG_ACT_RELU}


def basis_layout_for(plan: ChebPlan, N: int, Fin: int, K: int, Fout: int) -> str:
    """The layout a caller that keeps the basis to itself (the autograd
    functions below) should use: 'planes' where it applies (sample-major
    streaming path, Fin % 16 == 0: no basis-assembly pass), else 'rows'."""
    return "planes" if plan.basis_elems(N, Fin, K, Fout, "planes") else "rows"


def cheb_forward(plan: ChebPlan, x: torch.Tensor, W: torch.Tensor | None, K: int,
                 want_basis: bool = True, out_basis: torch.Tensor | None = None,
                 out_y: torch.Tensor | None = None, residual: torch.Tensor | None = None,
                 act: str = "none", layout: str = "rows"):
    """Basis (N*M, Fin*K) and y = act(basis @ W + residual) (N, M, Fout).
    W None -> basis only.  out_basis / out_y: pre-allocated contiguous outputs.
    layout: the basis layout ('rows' = lib/graph_conv.py:172; 'planes' =
    [K, N*M, Fin], see ChebRunner); pass the same one to the backward."""
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
    basis = y = None
    if need_basis:
        shape = (K, N * M, Fin) if layout == "planes" else (N * M, Fin * K)
        basis = out_basis if out_basis is not None else torch.empty(shape, device=dev,
                                                                    dtype=torch.float32)
        _check_out("out_basis", basis, (N * M, Fin * K))
    if W is not None:
        y = out_y if out_y is not None else torch.empty((N, M, Fout), device=dev, dtype=torch.float32)
        _check_out("out_y", y, (N * M * Fout,))
    if residual is not None:
        _check_dev("residual", residual)
        residual = residual.contiguous()
        if W is None or residual.numel() != N * M * Fout:
            raise ValueError(f"residual must be [N, M, Fout] = [{N}, {M}, {Fout}]")
    fwd_ws, _ = plan.workspace_bytes(N, Fin, K, Fout)
    ws, s = _plan_ws(plan, fwd_ws, x)
    _lib.call("cg_cheb_forward_layout", plan.handle, N, Fin, K, Fout, _p(x), _p(W), _p(residual),
              ACTS[act], _lib.BASIS_LAYOUTS[layout], _p(basis), _p(y), _p(ws), fwd_ws, s)
    return basis, y


def cheb_backward(plan: ChebPlan, dy: torch.Tensor, basis: torch.Tensor, W: torch.Tensor, K: int,
                  need_dx: bool = True, need_dW: bool = True, layout: str = "rows"):
    """(dx [N,M,Fin] or None, dW [Fin*K, Fout] or None); layout: the forward's."""
    _check_dev("dy", dy)
    dy = dy.contiguous()
    N, M, Fout = dy.shape
    FinK = int(W.shape[0])
    Fin = FinK // K
    dev = dy.device
    dx = torch.empty((N, M, Fin), device=dev, dtype=torch.float32) if need_dx else None
    dW = torch.empty((FinK, Fout), device=dev, dtype=torch.float32) if need_dW else None
    _, bwd_ws = plan.workspace_bytes(N, Fin, K, Fout)
    ws, s = _plan_ws(plan, bwd_ws, dy)
    _lib.call("cg_cheb_backward_layout", plan.handle, N, Fin, K, Fout, _p(dy), None,
              _lib.CG_ACT_NONE, _lib.BASIS_LAYOUTS[layout], _p(basis), _p(W.contiguous()), _p(dx),
              0, _p(dW), None, _p(ws), bwd_ws, s)
    return dx, dW


def cheb_backward_ex(plan: ChebPlan, dy: torch.Tensor, y: torch.Tensor | None, act: str,
                     basis: torch.Tensor, W: torch.Tensor, K: int, dx: torch.Tensor | None = None,
                     dx_accumulate: bool = False, need_dx: bool = True, need_dW: bool = True,
                     layout: str = "rows"):
    """Backward through y = act(basis W + residual): returns (dx, dW, dz) where
    dz = dy * act'(y) is also the gradient of the residual input.  With
    dx_accumulate the input gradient is added into the given ``dx``."""
    _check_dev("dy", dy)
    dy = dy.contiguous()
    N, M, Fout = dy.shape
    FinK = int(W.shape[0])
    Fin = FinK // K
    dev = dy.device
    if need_dx and dx is None:
        if dx_accumulate:
            raise ValueError("dx_accumulate needs a dx tensor")
        dx = torch.empty((N, M, Fin), device=dev, dtype=torch.float32)
    if dx is not None:
        _check_out("dx", dx, (N, M, Fin))
    dW = torch.empty((FinK, Fout), device=dev, dtype=torch.float32) if need_dW else None
    dz = torch.empty((N, M, Fout), device=dev, dtype=torch.float32)
    _, bwd_ws = plan.workspace_bytes(N, Fin, K, Fout)
    ws, s = _plan_ws(plan, bwd_ws, dy)
    _lib.call("cg_cheb_backward_layout", plan.handle, N, Fin, K, Fout, _p(dy), _p(y), ACTS[act],
              _lib.BASIS_LAYOUTS[layout], _p(basis), _p(W.contiguous()),
              _p(dx if need_dx else None), int(dx_accumulate), _p(dW), _p(dz), _p(ws), bwd_ws, s)
    return (dx if need_dx else None), dW, dz


def mse_loss(pred: torch.Tensor, labels: torch.Tensor, need_grad: bool = True):
    """lib/graph_model.py:255 mean((labels - pred)^2) on device: (loss [1], dpred or None)."""
    _check_dev("pred", pred)
    _check_dev("labels", labels)
    pred, labels = pred.contiguous(), labels.contiguous()
    if pred.numel() != labels.numel():
        raise ValueError("pred and labels differ in size")
    n = pred.numel()
    nb = ctypes.c_size_t()
    _lib.call("cg_mse_loss_workspace_bytes", n, ctypes.byref(nb))
    ws = torch.empty(max(nb.value, 1), device=pred.device, dtype=torch.uint8)
    loss = torch.empty((1,), device=pred.device, dtype=torch.float32)
    dpred = torch.empty_like(pred) if need_grad else None
    _lib.call("cg_mse_loss", _p(pred), _p(labels), n, _p(loss), _p(dpred), _p(ws), nb.value,
              _stream(pred))
    return loss, dpred


class ChebRunner:
    """Pre-allocated forward/backward of one (plan, N, Fin, K, Fout) shape:
    every device buffer (basis, y, dx, dW, workspace) is allocated once, so a
    step is just the C-ABI launches on the current stream -- no allocator or
    Python-side shape work per call (and safe to capture in a HIP graph).
    The forward's workspace is dead once the forward has run, so the forward
    and the backward share ONE buffer of max(fwd, bwd) bytes (config D at
    N = 256: 51.5 GB instead of 68.7 GB)."""

    def __init__(self, plan: ChebPlan, N: int, Fin: int, K: int, Fout: int, device,
                 basis_layout: str = "rows"):
        """basis_layout: 'rows' ([N*M, Fin*K], lib/graph_conv.py:172), 'orders'
        ([N, Fin*K, Mb], one plane per order: the fast forward stores it during
        the recurrence; Fin <= 2 fast path with fused dW only) or 'planes'
        ([K, N*M, Fin], T_k in the layout of x: the streaming steps write their
        own plane and skip the basis assembly; sample-major streaming path with
        Fin % 16 == 0 only).  The basis is
        this runner's saved tensor either way.  On config B the orders layout
        makes the forward ~1.3 us faster and the backward ~1.9 us slower
        (profiles/r02_orders), so 'rows' stays the default."""
        self.plan, self.N, self.Fin, self.K, self.Fout = plan, int(N), int(Fin), int(K), int(Fout)
        dev = torch.device(device)
        self.path = plan.query_path(N, Fin, K, Fout)
        fb, bb = plan.workspace_bytes(N, Fin, K, Fout)
        M = plan.M
        f32 = dict(device=dev, dtype=torch.float32)
        if basis_layout == "orders":
            if plan.basis_elems(N, Fin, K, Fout, "orders") is None:
                raise ValueError("orders basis layout does not apply to this shape "
                                 "(needs the fast forward and the fused-dW fast backward)")
            self.basis = torch.empty((N, Fin * K, (M + 31) // 32 * 32), **f32)
        elif basis_layout == "planes":
            if plan.basis_elems(N, Fin, K, Fout, "planes") is None:
                raise ValueError("planes basis layout does not apply to this shape (needs the "
                                 "sample-major streaming path, Fin % 16 == 0, K >= 2)")
            self.basis = torch.empty((K, N * M, Fin), **f32)
        elif basis_layout == "rows":
            self.basis = torch.empty((N * M, Fin * K), **f32)
        else:
            raise ValueError(f"unknown basis layout {basis_layout!r}")
        self.basis_layout = basis_layout
        self._lay = _lib.BASIS_LAYOUTS[basis_layout]
        self.y = torch.empty((N, M, Fout), **f32)
        self.dx = torch.empty((N, M, Fin), **f32)
        self.dW = torch.empty((Fin * K, Fout), **f32)
        self.ws = torch.empty(max(fb, bb, 1), device=dev, dtype=torch.uint8)
        self.fws = self.bws = self.ws
        self.fwd_bytes, self.bwd_bytes = fb, bb
        self._fwd = _lib.lib().cg_cheb_forward_layout
        self._bwd = _lib.lib().cg_cheb_backward_layout

    def input_plane(self) -> torch.Tensor | None:
        """Planes layout: plane 0 of the saved basis as an [N, M, Fin] tensor.  A
        producer that writes the filter input there (and passes it as x) saves
        the forward's copy of x into plane 0 (cg_cheb_forward_layout reads
        T_0 in place when x == basis).  None for the other layouts."""
        if self.basis_layout != "planes":
            return None
        return self.basis[0].view(self.N, self.plan.M, self.Fin)

    def basis_rows(self) -> torch.Tensor:
        """The saved basis as [N*M, Fin*K] (a copy when the layout is 'orders')."""
        if self.basis_layout == "rows":
            return self.basis
        if self.basis_layout == "planes":  # [K][N*M][Fin] -> column fin*K + k
            return self.basis.permute(1, 2, 0).reshape(self.N * self.plan.M, self.Fin * self.K)
        M = self.plan.M
        return self.basis[:, :, :M].permute(0, 2, 1).reshape(self.N * M, self.Fin * self.K)

    def forward(self, x: torch.Tensor, W: torch.Tensor, stream=None):
        s = stream if stream is not None else torch.cuda.current_stream(x.device).cuda_stream
        st = self._fwd(self.plan.handle, self.N, self.Fin, self.K, self.Fout, x.data_ptr(),
                       W.data_ptr(), None, 0, self._lay, self.basis.data_ptr(), self.y.data_ptr(),
                       self.fws.data_ptr(), self.fwd_bytes, s)
        _lib.check("cg_cheb_forward_layout", st)
        return self.y

    def forward_adam(self, x: torch.Tensor, W: torch.Tensor, grad: torch.Tensor, m: torch.Tensor,
                     v: torch.Tensor, W_out: torch.Tensor, m_out: torch.Tensor,
                     v_out: torch.Tensor, step: int, lr: float = 1e-3, beta1: float = 0.9,
                     beta2: float = 0.999, eps: float = 1e-8, grad_scale: float = 1.0,
                     stream=None):
        """The exchange step's Adam on W applied by the forward that consumes it
        (cg_cheb_forward_adam): W_out, m_out, v_out = ApplyAdam(W, grad; m, v),
        then y = chebyshev5(x; W_out).  Outputs out of place (double-buffer them)."""
        shape = (self.Fin * self.K, self.Fout)
        for name, t_ in (("W", W), ("grad", grad), ("m", m), ("v", v), ("W_out", W_out),
                         ("m_out", m_out), ("v_out", v_out)):
            _check_out(name, t_, shape)
        s = stream if stream is not None else torch.cuda.current_stream(x.device).cuda_stream
        st = _lib.lib().cg_cheb_forward_adam(
            self.plan.handle, self.N, self.Fin, self.K, self.Fout, x.data_ptr(), W.data_ptr(),
            grad.data_ptr(), m.data_ptr(), v.data_ptr(), lr, beta1, beta2, eps, step, grad_scale,
            W_out.data_ptr(), m_out.data_ptr(), v_out.data_ptr(), self._lay,
            self.basis.data_ptr(), self.y.data_ptr(), self.fws.data_ptr(), self.fwd_bytes, s)
        _lib.check("cg_cheb_forward_adam", st)
        return self.y

    def backward(self, dy: torch.Tensor, W: torch.Tensor, need_dx: bool = True, stream=None):
        s = stream if stream is not None else torch.cuda.current_stream(dy.device).cuda_stream
        st = self._bwd(self.plan.handle, self.N, self.Fin, self.K, self.Fout, dy.data_ptr(), None, 0,
                       self._lay, self.basis.data_ptr(), W.data_ptr(),
                       self.dx.data_ptr() if need_dx else None, 0, self.dW.data_ptr(), None,
                       self.bws.data_ptr(), self.bwd_bytes, s)
        _lib.check("cg_cheb_backward_layout", st)
        return (self.dx if need_dx else None), self.dW

    def backward_adam(self, dy: torch.Tensor, W: torch.Tensor, m: torch.Tensor, v: torch.Tensor,
                      step: int, lr: float = 1e-3, beta1: float = 0.9, beta2: float = 0.999,
                      eps: float = 1e-8, grad_scale: float = 1.0, need_dx: bool = True,
                      stream=None):
        """backward + Adam on W in place, the update fused into the dW reduction
        (cg_cheb_backward_adam_layout; one-GPU step, lib/graph_model.py:277-298)."""
        shape = (self.Fin * self.K, self.Fout)
        for name, t_ in (("W", W), ("m", m), ("v", v)):
            _check_out(name, t_, shape)   # updated in place for i < Fin*K*Fout
        if len({W.data_ptr(), m.data_ptr(), v.data_ptr(), self.dW.data_ptr()}) != 4:
            raise ValueError("backward_adam: W, m, v and dW must be distinct buffers")
        s = stream if stream is not None else torch.cuda.current_stream(dy.device).cuda_stream
        st = _lib.lib().cg_cheb_backward_adam_layout(
            self.plan.handle, self.N, self.Fin, self.K, self.Fout, self._lay, dy.data_ptr(),
            self.basis.data_ptr(), W.data_ptr(), self.dx.data_ptr() if need_dx else None,
            self.dW.data_ptr(), m.data_ptr(), v.data_ptr(), lr, beta1, beta2, eps, step,
            grad_scale, self.bws.data_ptr(), self.bwd_bytes, s)
        _lib.check("cg_cheb_backward_adam_layout", st)
        return (self.dx if need_dx else None), self.dW


def _saved_basis_layout(plan: ChebPlan, basis: torch.Tensor, layout: str, N: int, Fin: int, K: int,
                        Fout: int):
    """The basis an autograd backward hands to the C ABI: the saved one, or --
    when the plan's path / variant was changed between forward and backward so
    that the planes layout no longer applies -- the same values re-laid as
    the rows layout of lib/graph_conv.py:172 (column fin*K + k)."""
    if layout != "planes" or plan.basis_elems(N, Fin, K, Fout, "planes"):
        return basis, layout
    return basis.permute(1, 2, 0).reshape(N * plan.M, Fin * K).contiguous(), "rows"


class ChebConv(torch.autograd.Function):
    """y = chebyshev5(x; L~, W, K) with the HIP forward/backward kernels."""

    @staticmethod
    def forward(ctx, x, W, plan: ChebPlan, K: int):
        # the saved basis is internal: the planes layout where it applies
        lay = basis_layout_for(plan, x.shape[0], x.shape[2], K, W.shape[1])
        basis, y = cheb_forward(plan, x, W, K, want_basis=True, layout=lay)
        ctx.save_for_backward(basis, W)
        ctx.plan, ctx.K, ctx.layout = plan, K, lay
        return y

    @staticmethod
    def backward(ctx, dy):
        basis, W = ctx.saved_tensors
        N, Fout = dy.shape[0], W.shape[1]
        basis, lay = _saved_basis_layout(ctx.plan, basis, ctx.layout, N, W.shape[0] // ctx.K, ctx.K,
                                         Fout)
        dx, dW = cheb_backward(ctx.plan, dy, basis, W, ctx.K, need_dx=ctx.needs_input_grad[0],
                               layout=lay)
        return dx, dW, None, None


class ChebConvAct(torch.autograd.Function):
    """y = act(chebyshev5(x; L~, W, K) + residual) in one kernel pass
    (lib/graph_conv.py:256-262); residual may be None."""

    @staticmethod
    def forward(ctx, x, W, residual, plan: ChebPlan, K: int, act: str):
        lay = basis_layout_for(plan, x.shape[0], x.shape[2], K, W.shape[1])
        basis, y = cheb_forward(plan, x, W, K, want_basis=True, residual=residual, act=act,
                                layout=lay)
        ctx.save_for_backward(basis, W, y)
        ctx.plan, ctx.K, ctx.act, ctx.has_res = plan, K, act, residual is not None
        ctx.layout = lay
        return y

    @staticmethod
    def backward(ctx, dy):
        basis, W, y = ctx.saved_tensors
        basis, lay = _saved_basis_layout(ctx.plan, basis, ctx.layout, dy.shape[0],
                                         W.shape[0] // ctx.K, ctx.K, W.shape[1])
        dx, dW, dz = cheb_backward_ex(ctx.plan, dy, y, ctx.act, basis, W, ctx.K,
                                      need_dx=ctx.needs_input_grad[0], layout=lay)
        return dx, dW, (dz if ctx.has_res else None), None, None, None


def cheb_conv(x, W, plan: ChebPlan, K: int, residual=None, act: str = "none"):
    if residual is None and act == "none":
        return ChebConv.apply(x, W, plan, K)
    return ChebConvAct.apply(x, W, residual, plan, K, act)


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


def weight_grad(basis: torch.Tensor, dy: torch.Tensor, out: torch.Tensor | None = None,
                accumulate: bool = False) -> torch.Tensor:
    """dW = basis^T dy over all rows (basis [R, FinK], dy [R, Fout] in any
    [..., Fout] shape); accumulate=True adds into ``out``."""
    _check_dev("basis", basis)
    _check_dev("dy", dy)
    FinK = int(basis.shape[-1])
    R = basis.numel() // FinK
    Fout = int(dy.shape[-1])
    if dy.numel() != R * Fout:
        raise ValueError(f"dy has {dy.numel()} elements, expected R*Fout = {R * Fout}")
    if out is None:
        if accumulate:
            raise ValueError("accumulate=True needs an out tensor")
        out = torch.empty((FinK, Fout), device=basis.device, dtype=torch.float32)
    _check_out("out", out, (FinK, Fout))
    nb = ctypes.c_size_t()
    _lib.call("cg_weight_grad_workspace_bytes", R, FinK, Fout, ctypes.byref(nb))
    ws = torch.empty(max(nb.value, 1), device=basis.device, dtype=torch.uint8)
    _lib.call("cg_weight_grad", R, FinK, Fout, _p(basis.contiguous()), _p(dy.contiguous()), _p(out),
              int(accumulate), _p(ws), nb.value, _stream(basis))
    return out


def weight_grad_planes(planes: torch.Tensor, plane_stride: int, K: int, R: int, dy: torch.Tensor,
                       out: torch.Tensor | None = None, accumulate: bool = False) -> torch.Tensor:
    """dW [Fin*K, Fout] (row fin*K + k) = sum_k planes_k^T dy over R rows, the K
    planes [R, Fin] of ``planes``' storage plane_stride floats apart (plane k
    at planes.data_ptr() + k*plane_stride floats); one pass over dy."""
    _check_dev("planes", planes)
    _check_dev("dy", dy)
    Fin = int(planes.shape[-1])
    Fout = int(dy.shape[-1])
    if dy.numel() != R * Fout or not dy.is_contiguous():
        raise ValueError(f"dy must be a contiguous tensor of R*Fout = {R * Fout} elements")
    avail = planes.untyped_storage().nbytes() // 4 - planes.storage_offset()
    if plane_stride < R * Fin or avail < (K - 1) * plane_stride + R * Fin:
        raise ValueError("planes: storage too small for K planes at this stride")
    if out is None:
        if accumulate:
            raise ValueError("accumulate=True needs an out tensor")
        out = torch.empty((Fin * K, Fout), device=planes.device, dtype=torch.float32)
    _check_out("out", out, (Fin * K, Fout))
    nb = ctypes.c_size_t()
    _lib.call("cg_weight_grad_workspace_bytes", R, Fin * K, Fout, ctypes.byref(nb))
    ws = torch.empty(max(nb.value, 1), device=planes.device, dtype=torch.uint8)
    _lib.call("cg_weight_grad_planes", int(R), Fin, int(K), Fout, _p(planes), int(plane_stride),
              _p(dy), _p(out), int(accumulate), _p(ws), nb.value, _stream(planes))
    return out


def lstm_weight_grads(h_planes: torch.Tensor, h_plane_stride: int, x_planes: torch.Tensor,
                      x_plane_stride: int, K: int, R: int, dpre: torch.Tensor):
    """dWh [H*K, 4H], dWx [Fin*K, 4H] and db [4H] of a gconv-LSTM layer in ONE
    pass over dpre [R, 4H] (cg_lstm_weight_grads): the K h planes [R, H] of
    h_planes' storage h_plane_stride floats apart, the K x planes [R, Fin] of
    x_planes' storage likewise."""
    for name, t in (("h_planes", h_planes), ("x_planes", x_planes), ("dpre", dpre)):
        _check_dev(name, t)
    H, Fin = int(h_planes.shape[-1]), int(x_planes.shape[-1])
    if dpre.numel() != R * 4 * H or not dpre.is_contiguous():
        raise ValueError(f"dpre must be a contiguous tensor of R*4H = {R * 4 * H} elements")
    for name, t, st, w in (("h_planes", h_planes, h_plane_stride, H),
                           ("x_planes", x_planes, x_plane_stride, Fin)):
        avail = t.untyped_storage().nbytes() // 4 - t.storage_offset()
        if st < R * w or avail < (K - 1) * st + R * w:
            raise ValueError(f"{name}: storage too small for K planes at this stride")
    f32 = dict(device=dpre.device, dtype=torch.float32)
    dWh = torch.empty((H * K, 4 * H), **f32)
    dWx = torch.empty((Fin * K, 4 * H), **f32)
    db = torch.empty((4 * H,), **f32)
    nb = ctypes.c_size_t()
    _lib.call("cg_lstm_weight_grads_workspace_bytes", int(R), H, Fin, int(K), ctypes.byref(nb))
    ws = torch.empty(max(nb.value, 1), device=dpre.device, dtype=torch.uint8)
    _lib.call("cg_lstm_weight_grads", int(R), H, Fin, int(K), _p(h_planes), int(h_plane_stride),
              _p(x_planes), int(x_plane_stride), _p(dpre), _p(dWh), _p(dWx), _p(db), _p(ws),
              nb.value, _stream(dpre))
    return dWh, dWx, db


def bias_grad(dy: torch.Tensor, out: torch.Tensor | None = None, accumulate: bool = False):
    """db = dy summed over every axis but the last (gradient of a broadcast bias)."""
    _check_dev("dy", dy)
    C = int(dy.shape[-1])
    R = dy.numel() // C
    if out is None:
        if accumulate:
            raise ValueError("accumulate=True needs an out tensor")
        out = torch.empty((C,), device=dy.device, dtype=torch.float32)
    _check_out("out", out, (C,))
    nb = ctypes.c_size_t()
    _lib.call("cg_bias_grad_workspace_bytes", R, C, ctypes.byref(nb))
    ws = torch.empty(max(nb.value, 1), device=dy.device, dtype=torch.uint8)
    _lib.call("cg_bias_grad", R, C, _p(dy.contiguous()), _p(out), int(accumulate), _p(ws), nb.value,
              _stream(dy))
    return out


LSTM_GATES = {"reference": 0, "standard": 1}


def lstm_cell_forward(gx, gh, bias, c, H: int, gates="reference", out_c=None, out_h=None,
                      out_act=None):
    """Pointwise part of GConvLSTMCell (lib/gconv_lstm.py:183-221): gx, gh
    [..., 4H] gate pre-activations of the x- and h-conv (gh None = 0), bias
    [4H] (None = 0), c [..., H] (None = 0).  Returns (c', h', act [..., 4H])."""
    _check_dev("gx", gx)
    R = gx.numel() // (4 * H)
    lead = tuple(gx.shape[:-1])
    dev = gx.device
    for name, t, n in (("gh", gh, 4 * H), ("bias", bias, 4 * H), ("c", c, H)):
        if t is not None:
            _check_dev(name, t)
            if not t.is_contiguous() or t.numel() != (n if name == "bias" else R * n):
                raise ValueError(f"{name}: bad shape {tuple(t.shape)}")
    c_out = out_c if out_c is not None else torch.empty(lead + (H,), device=dev, dtype=torch.float32)
    h_out = out_h if out_h is not None else torch.empty(lead + (H,), device=dev, dtype=torch.float32)
    act = out_act if out_act is not None else torch.empty(lead + (4 * H,), device=dev,
                                                          dtype=torch.float32)
    _check_out("c_out", c_out, (R, H))
    _check_out("h_out", h_out, (R, H))
    _check_out("act", act, (R, 4 * H))
    _lib.call("cg_lstm_cell_forward", R, H, LSTM_GATES[gates], _p(gx.contiguous()), _p(gh), _p(bias),
              _p(c), _p(c_out), _p(h_out), _p(act), _stream(gx))
    return c_out, h_out, act


def lstm_hconv_supported(plan: ChebPlan, H: int, K: int) -> bool:
    """Whether cg_lstm_hconv_step serves this graph / hidden size / order."""
    ok = ctypes.c_int32()
    _lib.call("cg_lstm_hconv_supported", plan.handle, int(H), int(K), ctypes.byref(ok))
    return bool(ok.value)


def lstm_hconv_step(plan: ChebPlan, h_prev, c_prev, gx, Wh, bias, K: int, gates="reference",
                    out_c=None, out_h=None, out_act=None, planes=None, plane_stride: int = 0):
    """One time step of GConvLSTMCell's h path in one launch (cg_lstm_hconv_step):
    the Chebyshev basis of h_prev, gh = basis Wh on MFMA and the gate update,
    given the step's x-conv gx [..., 4H].  planes (optional, a tensor whose
    storage holds K-1 planes [N, M, H] plane_stride floats apart) receives
    T_1 .. T_{K-1} of h_prev.  Returns (c', h', act)."""
    _check_dev("h_prev", h_prev)
    h_prev = h_prev.contiguous()
    N, M, H = (int(v) for v in h_prev.shape)
    R = N * M
    dev = h_prev.device
    for name, t, n in (("gx", gx, 4 * H), ("c_prev", c_prev, H), ("bias", bias, 4 * H)):
        if t is not None:
            _check_dev(name, t)
            if not t.is_contiguous() or t.numel() != (n if name == "bias" else R * n):
                raise ValueError(f"{name}: bad shape {tuple(t.shape)}")
    if tuple(Wh.shape) != (K * H, 4 * H) or not Wh.is_contiguous():
        raise ValueError(f"Wh must be a contiguous [{K * H}, {4 * H}] tensor")
    c_out = out_c if out_c is not None else torch.empty((N, M, H), device=dev, dtype=torch.float32)
    h_out = out_h if out_h is not None else torch.empty((N, M, H), device=dev, dtype=torch.float32)
    act = out_act if out_act is not None else torch.empty((N, M, 4 * H), device=dev,
                                                          dtype=torch.float32)
    _check_out("c_out", c_out, (R, H))
    _check_out("h_out", h_out, (R, H))
    _check_out("act", act, (R, 4 * H))
    if planes is not None:
        _check_dev("planes", planes)
        need = (K - 2) * plane_stride + R * H if K > 1 else 0
        avail = planes.untyped_storage().nbytes() // 4 - planes.storage_offset()
        if K > 1 and (plane_stride < R * H or avail < need):
            raise ValueError("planes: storage too small for the K-1 planes at this stride")
        if planes.data_ptr() % 16 or (K > 1 and plane_stride % 4):
            raise ValueError("planes: needs a 16-byte aligned start and a stride that is a "
                             "multiple of 4 floats (the kernel stores float4)")
    if h_prev.data_ptr() % 16:
        h_prev = h_prev.clone()  # float4 loads: a view at an odd offset is copied
    _lib.call("cg_lstm_hconv_step", plan.handle, N, H, int(K), LSTM_GATES[gates], _p(h_prev),
              _p(c_prev), _p(gx), _p(Wh), _p(bias), _p(c_out), _p(h_out), _p(act), _p(planes),
              int(plane_stride), _stream(h_prev))
    return c_out, h_out, act


def lstm_cell_backward(dh, dh_rec, dc, act, c, c_out, H: int, gates="reference", out_dpre=None,
                       need_dc_prev=True):
    """Backward of lstm_cell_forward: (dpre [..., 4H], dc_prev [..., H] or None)."""
    _check_dev("act", act)
    _check_dev("c_out", c_out)
    R = act.numel() // (4 * H)
    dev = act.device
    for name, t in (("dh", dh), ("dh_rec", dh_rec), ("dc", dc), ("c", c)):
        if t is not None:
            _check_dev(name, t)
            if not t.is_contiguous() or t.numel() != R * H:
                raise ValueError(f"{name}: bad shape {tuple(t.shape)}")
    dpre = out_dpre if out_dpre is not None else torch.empty(tuple(act.shape), device=dev,
                                                             dtype=torch.float32)
    _check_out("dpre", dpre, (R, 4 * H))
    dc_prev = torch.empty(tuple(c_out.shape), device=dev, dtype=torch.float32) if need_dc_prev else None
    _lib.call("cg_lstm_cell_backward", R, H, LSTM_GATES[gates], _p(dh), _p(dh_rec), _p(dc), _p(act),
              _p(c), _p(c_out), _p(dpre), _p(dc_prev), _stream(act))
    return dpre, dc_prev


def lstm_seq_supported(plan: ChebPlan, H: int, K: int) -> bool:
    """Whether the one-launch layer forward (cg_lstm_seq_forward) and the
    one-launch BPTT step (cg_lstm_bwd_step) serve this graph / H / K."""
    ok = ctypes.c_int32()
    _lib.call("cg_lstm_seq_supported", plan.handle, int(H), int(K), ctypes.byref(ok))
    return bool(ok.value)


def lstm_seq_fault(plan: ChebPlan, wait: bool = True) -> bool | None:
    """The plan's sticky sequence-launch fault word (cg_lstm_seq_fault): raises
    CGError (and resets the word) if a pair hand-off of any k_lstm_seq launch
    so far timed out -- that launch's hs / cs / act then hold NaN from the lost
    step on.  wait=True blocks until the last launch has completed and returns
    False; wait=False never blocks and returns None while it is in flight."""
    f = ctypes.c_int32()
    _lib.call("cg_lstm_seq_fault", plan.handle, int(bool(wait)), 1, ctypes.byref(f))
    return None if f.value < 0 else False


def lstm_seq_forward(plan: ChebPlan, gx, Wh, bias, K: int, T: int, N: int, gates="reference",
                     h0=None, c0=None, out_hs=None, out_cs=None, out_act=None, planes=None,
                     plane_stride: int = 0, check: bool = False):
    """All T steps of a gconv-LSTM layer in ONE launch (cg_lstm_seq_forward):
    gx [T, N, M, 4H] (the x-conv of every step), h0 / c0 [N, M, H] or None
    (zero state).  planes (optional; a tensor whose storage holds K-1 planes
    [T, N, M, H] plane_stride floats apart) receives T_k of h_{t-1}, k >= 1.
    check=True waits for the launch and raises CGError if a pair hand-off timed
    out (lstm_seq_fault); without it the fault surfaces at the next check.
    Returns (hs [T, N, M, H], cs [T, N, M, H], act or None) -- act UNIT-major,
    [T, N, M, 4H] holding act[..., 4u + g] (g = z, i, f, o): lstm_bwd_step
    reads it with act_unit_major=True."""
    _check_dev("gx", gx)
    H = int(Wh.shape[1]) // 4
    M = plan.M
    R = T * N * M
    if not gx.is_contiguous() or gx.numel() != R * 4 * H:
        raise ValueError(f"gx must be a contiguous [{T}, {N}, {M}, {4 * H}] tensor")
    if tuple(Wh.shape) != (K * H, 4 * H) or not Wh.is_contiguous():
        raise ValueError(f"Wh must be a contiguous [{K * H}, {4 * H}] tensor")
    dev = gx.device
    for name, t, n in (("bias", bias, 4 * H), ("h0", h0, N * M * H), ("c0", c0, N * M * H)):
        if t is not None:
            _check_dev(name, t)
            if not t.is_contiguous() or t.numel() != n or t.data_ptr() % 16:
                raise ValueError(f"{name}: need a contiguous 16-byte aligned tensor of {n} floats")
    f32 = dict(device=dev, dtype=torch.float32)
    hs = out_hs if out_hs is not None else torch.empty((T, N, M, H), **f32)
    cs = out_cs if out_cs is not None else torch.empty((T, N, M, H), **f32)
    _check_out("hs", hs, (R, H))
    _check_out("cs", cs, (R, H))
    if out_act is not None:
        _check_out("act", out_act, (R, 4 * H))
    if planes is None and K > 1:  # the kernel hands Chebyshev orders through them
        planes = torch.empty((K - 1, R, H), **f32)
        plane_stride = R * H
    if planes is not None:
        _check_dev("planes", planes)
        need = (K - 2) * plane_stride + R * H if K > 1 else 0
        avail = planes.untyped_storage().nbytes() // 4 - planes.storage_offset()
        if K > 1 and (plane_stride < R * H or avail < need or planes.data_ptr() % 16
                      or plane_stride % 4):
            raise ValueError("planes: storage too small / misaligned for the K-1 planes")
    nb = ctypes.c_size_t()
    _lib.call("cg_lstm_seq_workspace_bytes", plan.handle, int(N), ctypes.byref(nb))
    ws = torch.empty(int(nb.value), device=dev, dtype=torch.uint8)
    s = _stream(gx)
    _lib.call("cg_lstm_seq_forward", plan.handle, int(T), int(N), int(H), int(K), LSTM_GATES[gates],
              _p(gx), _p(Wh), _p(bias), _p(h0), _p(c0), _p(hs), _p(cs), _p(out_act), _p(planes),
              int(plane_stride), _p(ws), int(nb.value), s)
    if check:
        lstm_seq_fault(plan, wait=True)
    return hs, cs, out_act


def lstm_seq_x_supported(plan: ChebPlan, Fin: int, H: int, K: int) -> bool:
    """Whether cg_lstm_seq_forward_x (the x-conv fused in) serves feat_in = Fin."""
    ok = ctypes.c_int32()
    _lib.call("cg_lstm_seq_x_supported", plan.handle, int(Fin), int(H), int(K), ctypes.byref(ok))
    return bool(ok.value)


def lstm_seq_forward_x(plan: ChebPlan, xs, Wx, Wh, bias, K: int, gates="reference", h0=None,
                       c0=None, out_hs=None, out_cs=None, out_act=None, planes=None,
                       plane_stride: int = 0, xplanes=None, check: bool = False):
    """lstm_seq_forward with the x-conv fused in (cg_lstm_seq_forward_x; feat_in
    <= 8): xs [T, N, M, F] instead of gx.  xplanes (optional, [K, T, N*M, F]):
    receives the x basis T_k(x_t), k = 0..K-1.  Returns (hs, cs, act, xplanes)."""
    _check_dev("xs", xs)
    xs = xs.contiguous()
    T, N, M, F = (int(v) for v in xs.shape)
    H = int(Wh.shape[1]) // 4
    R = T * N * M
    dev = xs.device
    f32 = dict(device=dev, dtype=torch.float32)
    if tuple(Wx.shape) != (K * F, 4 * H) or not Wx.is_contiguous():
        raise ValueError(f"Wx must be a contiguous [{K * F}, {4 * H}] tensor")
    if tuple(Wh.shape) != (K * H, 4 * H) or not Wh.is_contiguous():
        raise ValueError(f"Wh must be a contiguous [{K * H}, {4 * H}] tensor")
    for name, t, n in (("bias", bias, 4 * H), ("h0", h0, N * M * H), ("c0", c0, N * M * H)):
        if t is not None:
            _check_dev(name, t)
            if not t.is_contiguous() or t.numel() != n or t.data_ptr() % 16:
                raise ValueError(f"{name}: need a contiguous 16-byte aligned tensor of {n} floats")
    hs = out_hs if out_hs is not None else torch.empty((T, N, M, H), **f32)
    cs = out_cs if out_cs is not None else torch.empty((T, N, M, H), **f32)
    _check_out("hs", hs, (R, H))
    _check_out("cs", cs, (R, H))
    if out_act is not None:
        _check_out("act", out_act, (R, 4 * H))
    if planes is None and K > 1:
        planes = torch.empty((K - 1, R, H), **f32)
        plane_stride = R * H
    if planes is not None:
        _check_dev("planes", planes)
        need = (K - 2) * plane_stride + R * H if K > 1 else 0
        avail = planes.untyped_storage().nbytes() // 4 - planes.storage_offset()
        if K > 1 and (plane_stride < R * H or avail < need or planes.data_ptr() % 16
                      or plane_stride % 4):
            raise ValueError("planes: storage too small / misaligned for the K-1 planes")
    if xplanes is None:
        xplanes = torch.empty((K, R, F), **f32)
    _check_out("xplanes", xplanes, (K * R * F,))
    nb = ctypes.c_size_t()
    _lib.call("cg_lstm_seq_workspace_bytes", plan.handle, int(N), ctypes.byref(nb))
    ws = torch.empty(int(nb.value), device=dev, dtype=torch.uint8)
    s = _stream(xs)
    _lib.call("cg_lstm_seq_forward_x", plan.handle, T, N, F, int(H), int(K), LSTM_GATES[gates],
              _p(xs), _p(Wx), _p(xplanes), R * F, _p(Wh), _p(bias), _p(h0), _p(c0), _p(hs), _p(cs),
              _p(out_act), _p(planes), int(plane_stride), _p(ws), int(nb.value), s)
    if check:
        lstm_seq_fault(plan, wait=True)
    return hs, cs, out_act, xplanes


def lstm_bwd_step(plan: ChebPlan, dh, dh_rec, dc, act, c_prev, c_out, Wh, K: int,
                  gates="reference", out_dpre=None, need_dc_prev=True, out_dh_prev=None,
                  act_unit_major=False, need_dh_prev=True):
    """One BPTT step of a gconv-LSTM layer in ONE launch (cg_lstm_bwd_step):
    dpre = the gradient of the gate pre-activations, dc_prev, and dh_prev =
    the h-conv's input gradient.  dh / dh_rec / dc / c_prev may be None (= 0).
    act: gate-major [..., 4H] (lstm_cell_forward / lstm_hconv_step) or, with
    act_unit_major, the unit-major [..., H, 4] records of lstm_seq_forward*.
    need_dh_prev=False: the step ran no h-conv (step 0 of a zero-state layer):
    the pointwise backward only, dh_prev None.
    Returns (dpre [..., 4H], dc_prev [..., H] or None, dh_prev [..., H] or None)."""
    _check_dev("act", act)
    _check_dev("c_out", c_out)
    H = int(Wh.shape[1]) // 4
    R = act.numel() // (4 * H)
    N = R // plan.M
    dev = act.device
    for name, t in (("dh", dh), ("dh_rec", dh_rec), ("dc", dc), ("c_prev", c_prev),
                    ("c_out", c_out)):
        if t is not None:
            _check_dev(name, t)
            if not t.is_contiguous() or t.numel() != R * H or t.data_ptr() % 16:
                raise ValueError(f"{name}: bad shape / alignment {tuple(t.shape)}")
    if not act.is_contiguous() or act.data_ptr() % 16:
        raise ValueError("act: need a contiguous 16-byte aligned tensor")
    if tuple(Wh.shape) != (K * H, 4 * H) or not Wh.is_contiguous():
        raise ValueError(f"Wh must be a contiguous [{K * H}, {4 * H}] tensor")
    f32 = dict(device=dev, dtype=torch.float32)
    dpre = out_dpre if out_dpre is not None else \
        torch.empty(tuple(c_out.shape[:-1]) + (4 * H,), **f32)
    _check_out("dpre", dpre, (R, 4 * H))
    dc_prev = torch.empty(tuple(c_out.shape), **f32) if need_dc_prev else None
    dh_prev = None
    if need_dh_prev:
        dh_prev = out_dh_prev if out_dh_prev is not None else torch.empty(tuple(c_out.shape), **f32)
        _check_out("dh_prev", dh_prev, (R, H))
    _lib.call("cg_lstm_bwd_step", plan.handle, int(N), int(H), int(K), LSTM_GATES[gates], _p(dh),
              _p(dh_rec), _p(dc), _p(act), int(bool(act_unit_major)), _p(c_prev), _p(c_out), _p(Wh),
              _p(dpre), _p(dc_prev),
              _p(dh_prev), _stream(act))
    return dpre, dc_prev, dh_prev


class _Dropout(torch.autograd.Function):
    """tf.nn.dropout (TF 1.x) as DropoutWrapper applies it to a cell's outputs
    (lib/gconv_lstm.py:616, :623): cg_dropout_forward / cg_dropout_backward,
    the mask regenerated from ``seed`` in the backward."""

    @staticmethod
    def forward(ctx, x, keep_prob: float, seed: int):
        _check_dev("x", x)
        x = x.contiguous()
        y = torch.empty_like(x)
        _lib.call("cg_dropout_forward", _p(x), x.numel(), float(keep_prob), int(seed), _p(y), _stream(x))
        ctx.keep, ctx.seed = float(keep_prob), int(seed)
        return y

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        _lib.call("cg_dropout_backward", _p(dy), dy.numel(), ctx.keep, ctx.seed, _p(dx), _stream(dy))
        return dx, None, None


DROP_WEYL = 0x9E3779B97F4A7C15  # the mask draw's Weyl increment (epilogue.hip drop_u)


def dropout(x, keep_prob: float, seed: int, offset: int = 0):
    """y = (x / keep_prob) * floor(keep_prob + u), u ~ U[0,1) per element from
    (seed, index); keep_prob == 1 returns x.

    offset: x is the slice starting at element ``offset`` of a larger tensor
    dropped out under ``seed`` -- element i draws as element offset + i would
    there (the draw hashes seed + DROP_WEYL * (index + 1), so the offset folds
    into the seed: the same mask bits, no wider ABI)."""
    if int(offset) < 0:
        raise ValueError("dropout offset must be >= 0")
    if keep_prob >= 1.0:
        return x
    s = (int(seed) + DROP_WEYL * int(offset)) & ((1 << 64) - 1)
    return _Dropout.apply(x, keep_prob, s)


def clip_by_norm_(grads, clip_norm: float, check_numerics: bool = True):
    """tf.clip_by_norm + tf.check_numerics per gradient tensor, in place
    (gconvRNN.Model._build_optim, lib/gconvRNN.py:392-402): each g becomes
    (g * clip_norm) / max(||g||, clip_norm); with check_numerics a NaN / Inf
    in any clipped gradient raises FloatingPointError (one sync at the end)."""
    flag = None
    for g in grads:
        _check_dev("grad", g)
        if not g.is_contiguous():
            raise ValueError("clip_by_norm_: gradients must be contiguous")
        if flag is None:
            flag = torch.zeros((1,), device=g.device, dtype=torch.int32)
        _lib.call("cg_clip_by_norm", _p(g), g.numel(), float(clip_norm),
                  _p(flag) if check_numerics else None, _stream(g))
    if check_numerics and flag is not None and int(flag.item()):
        raise FloatingPointError("Numerical error in gradient (check_numerics after clip_by_norm)")
    return grads


def adam_update(param, grad, m, v, step: int, lr=1e-3, beta1=0.9, beta2=0.999, eps=1e-8,
                grad_scale=1.0):
    """In-place TF-1.x Adam step on device (lib/graph_model.py:293)."""
    for name, t in (("param", param), ("grad", grad), ("m", m), ("v", v)):
        _check_dev(name, t)
        if not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")
    _lib.call("cg_adam_update", _p(param), _p(grad), _p(m), _p(v), param.numel(), float(lr),
              float(beta1), float(beta2), float(eps), int(step), float(grad_scale), _stream(param))


def sgd_update(param, grad, lr=1e-3, grad_scale=1.0):
    """In-place tf.train.GradientDescentOptimizer step (lib/gconvRNN.py:383-384)."""
    for name, t in (("param", param), ("grad", grad)):
        _check_dev(name, t)
        if not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")
    _lib.call("cg_sgd_update", _p(param), _p(grad), param.numel(), float(lr), float(grad_scale),
              _stream(param))


def rmsprop_update(param, grad, ms, mom, lr=1e-3, rho=0.9, momentum=0.0, eps=1e-10,
                   grad_scale=1.0):
    """In-place tf.train.RMSPropOptimizer step (lib/gconvRNN.py:387-388; TF 1.x
    ApplyRMSProp, not centered).  ms starts at ONES, mom at zeros (TF 1.x slots)."""
    for name, t in (("param", param), ("grad", grad), ("ms", ms), ("mom", mom)):
        _check_dev(name, t)
        if not t.is_contiguous():
            raise ValueError(f"{name} must be contiguous")
    _lib.call("cg_rmsprop_update", _p(param), _p(grad), _p(ms), _p(mom), param.numel(), float(lr),
              float(rho), float(momentum), float(eps), float(grad_scale), _stream(param))


# -- bias + activation (lib/graph_conv.py:178-199, fc :220-226) --------------------
BIAS_ACTS = {"none": _lib.CG_ACT_NONE, "relu": _lib.CG_ACT_RELU, "tanh": _lib.CG_ACT_TANH}


class _BiasAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias, act: str):
        _check_dev("x", x)
        x = x.contiguous()
        n = x.numel()
        blen = 1
        if bias is not None:
            _check_dev("bias", bias)
            bias = bias.contiguous()
            blen = bias.numel()
            if n % blen:
                raise ValueError(f"bias of {blen} elements does not tile x of {n}")
        y = torch.empty_like(x)
        _lib.call("cg_bias_act_forward", n, blen, _p(x), _p(bias), BIAS_ACTS[act], _p(y), _stream(x))
        ctx.save_for_backward(y)
        ctx.act, ctx.blen, ctx.has_bias = act, blen, bias is not None
        ctx.bshape = None if bias is None else tuple(bias.shape)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dy = dy.contiguous()
        n = dy.numel()
        dz = torch.empty_like(dy)
        db = ws = None
        nb = 0
        if ctx.has_bias and ctx.needs_input_grad[1]:
            db = torch.empty(ctx.bshape, device=dy.device, dtype=torch.float32)
            b = ctypes.c_size_t()
            _lib.call("cg_bias_act_workspace_bytes", n, ctx.blen, ctypes.byref(b))
            nb = b.value
            ws = torch.empty(max(nb, 1), device=dy.device, dtype=torch.uint8)
        _lib.call("cg_bias_act_backward", n, ctx.blen, _p(dy), _p(y), BIAS_ACTS[ctx.act], _p(dz), _p(db),
                  0, _p(ws), nb, _stream(dy))
        return dz, db, None


def bias_act(x, bias=None, act: str = "relu"):
    """act(x + bias) with bias broadcast over the leading axes (bias [F] or
    [1,1,F]: one per filter; [1,M,F]: one per vertex and filter)."""
    return _BiasAct.apply(x, bias, act)


# -- plain GEMM on MFMA (the tf.matmul of fc / the Fourier transforms) -----------
def gemm(a: torch.Tensor, b: torch.Tensor, trans_a: bool = False, trans_b: bool = False,
         out: torch.Tensor | None = None) -> torch.Tensor:
    """op(a) @ op(b) for 2-D fp32 device tensors (cg_gemm_f32)."""
    _check_dev("a", a)
    _check_dev("b", b)
    a, b = a.contiguous(), b.contiguous()
    M, K = (a.shape[1], a.shape[0]) if trans_a else (a.shape[0], a.shape[1])
    Kb, N = (b.shape[1], b.shape[0]) if trans_b else (b.shape[0], b.shape[1])
    if K != Kb:
        raise ValueError(f"gemm: inner dimensions differ ({K} vs {Kb})")
    if out is None:
        out = torch.empty((M, N), device=a.device, dtype=torch.float32)
    _check_out("out", out, (M, N))
    _lib.call("cg_gemm_f32", int(trans_a), int(trans_b), M, N, K, _p(a), a.shape[1], _p(b), b.shape[1],
              _p(out), N, _stream(a))
    return out


class _MatMul(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        ctx.save_for_backward(a, b)
        return gemm(a, b)

    @staticmethod
    def backward(ctx, dc):
        a, b = ctx.saved_tensors
        da = gemm(dc, b, trans_b=True) if ctx.needs_input_grad[0] else None
        db = gemm(a, dc, trans_a=True) if ctx.needs_input_grad[1] else None
        return da, db


def matmul(a, b):
    """tf.matmul(a, b) for 2-D operands with its gradient, on the HIP GEMM."""
    return _MatMul.apply(a, b)


# -- Fourier filter (lib/graph_conv.py:83-111) ----------------------------------------
class _Fourier(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, U):
        for name, t in (("x", x), ("W", W), ("U", U)):
            _check_dev(name, t)
        x, W, U = x.contiguous(), W.contiguous(), U.contiguous()
        N, M, Fin = (int(s) for s in x.shape)
        if tuple(W.shape[::2]) != (M, Fin) or tuple(U.shape) != (M, M):
            raise ValueError(f"fourier: need W [M, Fout, Fin] = [{M}, *, {Fin}] and U [{M}, {M}], "
                             f"got {tuple(W.shape)} and {tuple(U.shape)}")
        Fout = int(W.shape[1])
        fb, bb = ctypes.c_size_t(), ctypes.c_size_t()
        _lib.call("cg_fourier_workspace_bytes", N, M, Fin, Fout, ctypes.byref(fb), ctypes.byref(bb))
        xhat = torch.empty((N, Fin, M), device=x.device, dtype=torch.float32)
        y = torch.empty((N, M, Fout), device=x.device, dtype=torch.float32)
        ws = torch.empty(max(fb.value, 1), device=x.device, dtype=torch.uint8)
        _lib.call("cg_fourier_forward", N, M, Fin, Fout, _p(U), _p(W), _p(x), _p(xhat), _p(y), _p(ws),
                  fb.value, _stream(x))
        ctx.save_for_backward(xhat, W, U)
        ctx.shape, ctx.bwd_bytes = (N, M, Fin, Fout), bb.value
        return y

    @staticmethod
    def backward(ctx, dy):
        xhat, W, U = ctx.saved_tensors
        N, M, Fin, Fout = ctx.shape
        dy = dy.contiguous()
        dx = torch.empty((N, M, Fin), device=dy.device, dtype=torch.float32) \
            if ctx.needs_input_grad[0] else None
        dW = torch.empty_like(W) if ctx.needs_input_grad[1] else None
        ws = torch.empty(max(ctx.bwd_bytes, 1), device=dy.device, dtype=torch.uint8)
        _lib.call("cg_fourier_backward", N, M, Fin, Fout, _p(U), _p(W), _p(xhat), _p(dy), _p(dx), _p(dW),
                  _p(ws), ctx.bwd_bytes, _stream(dy))
        return dx, dW, None


def fourier_conv(x, W, U):
    """filter_in_fourier (lib/graph_conv.py:83-99): x [N, M, Fin], W [M, Fout,
    Fin], U [M, M] (eigenvectors in columns, device fp32) -> [N, M, Fout]."""
    return _Fourier.apply(x, W, U)


# -- stacked-input ResGNN pieces (lib/graph_conv.py:272-303) -----------------------
class _SliceChannels(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, c0: int, c1: int):
        _check_dev("x", x)
        x = x.contiguous()
        C = int(x.shape[-1])
        rows = x.numel() // C
        out = torch.empty(tuple(x.shape[:-1]) + (c1 - c0,), device=x.device, dtype=torch.float32)
        _lib.call("cg_slice_channels", _p(x), rows, C, int(c0), int(c1), _p(out), _stream(x))
        ctx.shape, ctx.c0, ctx.c1 = tuple(x.shape), c0, c1
        return out

    @staticmethod
    def backward(ctx, dy):
        raise RuntimeError("slice_channels: the input channels are data (no gradient), "
                           "as in lib/graph_conv.py:274-303")


def slice_channels(x, c0: int, c1: int):
    """x[..., c0:c1] of a [N, M, C] device tensor as a new contiguous tensor
    (the reshape / unstack / concat of lib/graph_conv.py:281-286)."""
    return _SliceChannels.apply(x, int(c0), int(c1))


class _StackMerge(torch.autograd.Function):
    @staticmethod
    def forward(ctx, out_i, w_i, acc):
        for name, t in (("out_i", out_i), ("w_i", w_i)):
            _check_dev(name, t)
        out_i, w_i = out_i.contiguous(), w_i.contiguous()
        N, M, F = (int(s) for s in out_i.shape)
        if tuple(w_i.shape) != (M, F):
            raise ValueError(f"merge weight must be [{M}, {F}], got {tuple(w_i.shape)}")
        y = torch.empty_like(out_i)
        if acc is not None:
            y.copy_(acc)  # (buffer plumbing: the kernel accumulates into y)
        _lib.call("cg_stack_merge_forward", N, M, F, _p(out_i), _p(w_i), int(acc is not None), _p(y),
                  _stream(out_i))
        ctx.save_for_backward(out_i, w_i)
        ctx.has_acc = acc is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        out_i, w_i = ctx.saved_tensors
        dy = dy.contiguous()
        N, M, F = (int(s) for s in out_i.shape)
        d_o = torch.empty_like(out_i) if ctx.needs_input_grad[0] else None
        dw = torch.empty_like(w_i) if ctx.needs_input_grad[1] else None
        if d_o is not None or dw is not None:
            _lib.call("cg_stack_merge_backward", N, M, F, _p(dy), _p(out_i), _p(w_i), _p(d_o), _p(dw),
                      _stream(dy))
        return d_o, dw, (dy if ctx.has_acc else None)


def stack_merge(out_i, w_i, acc=None):
    """acc + relu(out_i) * w_i (w_i [M, F] broadcast over N; acc None: no add)
    -- one term of X = sum_i relu(net_i) * w_i, lib/graph_conv.py:292-301."""
    return _StackMerge.apply(out_i, w_i, acc)
