"""gconv-LSTM on the HIP Chebyshev path: drop-in for ``lib/gconv_lstm.py``'s
``GConvLSTMCell`` (lib/gconv_lstm.py:29-221) and the ``static_rnn`` over a
``MultiRNNCell`` that ``GconvModel.glstm_layer`` builds (:609-627).

Reference behaviour kept:
  * eight ``cheby_conv`` weights ``W{z,i,f,o}{x,h}t`` of shape [K*feat_in, H]
    and [K*H, H], ``random_uniform(-0.1, 0.1)`` (:98-115), and four biases
    ``b{z,i,f,o}t`` [H] with ``tf.get_variable``'s default (Glorot-uniform)
    initialiser (:173-176); ``K`` defaults to 2 (:95-96);
  * gate functions z = tan, i = f = sigmoid, o = tanh (:188, :195, :202, :209)
    -- ``gates="standard"`` gives the usual tanh / sigmoid instead;
  * ``forget_bias`` is accepted and ignored, as in the reference (:49);
  * ``__call__(inputs, state) -> (new_h, LSTMStateTuple(new_c, new_h))``.
  * ``DropoutWrapper(cell, output_keep_prob)`` (:616, :623): the cell's outputs
    go through ``tf.nn.dropout`` on a HIP kernel (``ops.dropout``); every
    wrapper draws its own mask stream (a distinct seed per wrapper unless one
    is given), as each TF DropoutWrapper owns an independent random op.
  * ``GLSTMModel``: ``inference_glstm`` (:271-281) -- glstm_layer, the last
    step's output, ``fc_layer`` (:629-636) -- with the MSE loss and the
    optimizer step (lib/graph_model.py:246-310; sgd / rmsprop of
    lib/gconvRNN.py:381-389), data parallel with ONE all-reduce of a flat
    gradient bucket per step (config E: batch 512 over 4 GPUs).

Run validation / inference under ``torch.no_grad()``: with gradients enabled a
lost pair hand-off of the one-launch layer is reported when the backward runs
(or at the next layer() call on the plan), not before the forward returns.

MI355X design: the four x-weights (and the four h-weights) are stored
concatenated as one [K*F, 4H] matrix, so a cell step is ONE x-conv plus ONE
h-step, not the reference's eight filters.  With H = 32 on graphs of up to
1024 vertices (config E) the h-step is a single launch
(``cg_lstm_hconv_step``): the Chebyshev basis of h in LDS, the gate
contraction on MFMA and the gate update in its epilogue (``hconv="fused"``);
otherwise it is a chebyshev5 call plus the pointwise kernel.  ``static_rnn``
additionally batches the x-conv of ALL time steps into one call (it does not
depend on the recurrence), runs the T h-steps back to back, and in the
backward sums the h-weight gradient of all steps per Chebyshev order with one
``cg_weight_grad`` over the stacked steps.
"""
from __future__ import annotations

import collections
import math

import torch

import ctypes
import itertools

from . import _lib
from . import ops
from .graph_conv import truncated_normal_
from .plan import plan_for

# distinct default mask streams per DropoutWrapper (TF: one random op each)
_DROPOUT_ORDINAL = itertools.count(1)

_LSTMStateTuple = collections.namedtuple("LSTMStateTuple", ("c", "h"))


class LSTMStateTuple(_LSTMStateTuple):
    """(c, h) -- lib/gconv_lstm.py:16-26."""
    __slots__ = ()

    @property
    def dtype(self):
        c, h = self
        if c.dtype != h.dtype:
            raise TypeError("Inconsistent internal state")
        return c.dtype


GATE_NAMES = ("z", "i", "f", "o")


class GConvLSTMCell:
    """lib/gconv_lstm.py:29-221 on the HIP kernels.  Parameters live in
    ``Wx`` [K*feat_in, 4H], ``Wh`` [K*H, 4H], ``b`` [4H]; ``variables`` maps the
    reference's variable names (``Wzxt``, ``Wiht``, ``bft``, ...) to views."""

    def __init__(self, num_units, forget_bias=1.0, state_is_tuple=True, activation=None,
                 reuse=None, laplacian=None, lmax=None, K=None, feat_in=None, nNode=None,
                 filter_type="cheby_conv", gates="reference", device=None, generator=None,
                 hconv="auto"):
        if filter_type != "cheby_conv":
            raise NotImplementedError(f"filter_type={filter_type!r}: only the Chebyshev filter "
                                      "is on the MI355X path (fourier_conv is out of scope)")
        if laplacian is None or feat_in is None:
            raise ValueError("laplacian and feat_in are required")
        if gates not in ops.LSTM_GATES:
            raise ValueError(f"gates must be one of {list(ops.LSTM_GATES)}")
        self._num_units = H = int(num_units)
        self._forget_bias = forget_bias          # unused, as in the reference
        self._state_is_tuple = state_is_tuple
        self._laplacian = laplacian
        self._lmax = 2 if lmax is None else lmax  # graph.lmax(normalized L) == 2
        self._K = 2 if K is None else int(K)      # :95-96
        self._feat_in = int(feat_in)
        self._nNode = int(nNode) if nNode is not None else int(laplacian.shape[0])
        self.gates = gates
        self.device = torch.device(device if device is not None else "cuda")
        dev_index = self.device.index if self.device.index is not None else 0
        self.plan = plan_for(laplacian, lmax=self._lmax, device=dev_index)
        K, F = self._K, self._feat_in
        f32 = dict(device=self.device, dtype=torch.float32)
        with torch.no_grad():
            Wx = torch.empty((K * F, 4 * H), **f32).uniform_(-0.1, 0.1, generator=generator)
            Wh = torch.empty((K * H, 4 * H), **f32).uniform_(-0.1, 0.1, generator=generator)
            lim = math.sqrt(6.0 / (H + H))  # glorot_uniform of a [H] vector: fan_in = fan_out = H
            b = torch.empty((4 * H,), **f32).uniform_(-lim, lim, generator=generator)
        self.Wx = torch.nn.Parameter(Wx)
        self.Wh = torch.nn.Parameter(Wh)
        self.b = torch.nn.Parameter(b)
        # h path: "seq" = the whole layer's T steps in one launch
        # (cg_lstm_seq_forward) and one launch per BPTT step (cg_lstm_bwd_step);
        # "fused" = one launch per forward step (cg_lstm_hconv_step); "unfused"
        # = chebyshev5 + pointwise kernel; "auto" picks the first that applies
        if hconv not in ("auto", "seq", "fused", "unfused"):
            raise ValueError("hconv must be 'auto', 'seq', 'fused' or 'unfused'")
        supported = ops.lstm_hconv_supported(self.plan, H, self._K)
        seq_ok = ops.lstm_seq_supported(self.plan, H, self._K)
        if hconv == "fused" and not supported:
            raise ValueError(f"hconv='fused' needs H = 32 and M <= 1024 (H={H}, M={self.plan.M})")
        if hconv == "seq" and not seq_ok:
            raise ValueError(f"hconv='seq' needs H = 32, M <= 1024, K <= 4 and L~ in LDS "
                             f"(H={H}, M={self.plan.M}, K={self._K})")
        self.seq = seq_ok and hconv in ("auto", "seq")
        # feat_in <= 8: the x-conv runs inside the sequence kernel too
        self.seq_x = self.seq and ops.lstm_seq_x_supported(self.plan, self._feat_in, H, self._K)
        self.fused = supported and hconv != "unfused"

    # -- reference properties ---------------------------------------------------
    @property
    def state_size(self):
        if self._state_is_tuple:
            return LSTMStateTuple((self._nNode, self._num_units), (self._nNode, self._num_units))
        return 2 * self._num_units

    @property
    def output_size(self):
        return self._num_units

    @property
    def variables(self):
        H = self._num_units
        v = {}
        for q, g in enumerate(GATE_NAMES):
            sl = slice(q * H, (q + 1) * H)
            v[f"W{g}xt"] = self.Wx[:, sl]
            v[f"W{g}ht"] = self.Wh[:, sl]
            v[f"b{g}t"] = self.b[sl]
        return v

    def parameters(self):
        return [self.Wx, self.Wh, self.b]

    def zero_state(self, batch_size, dtype=torch.float32):
        """(c, h) zeros of [batch, nNode, H] (lib/gconv_lstm.py:71-76)."""
        shape = (int(batch_size), self._nNode, self._num_units)
        return (torch.zeros(shape, device=self.device, dtype=dtype),
                torch.zeros(shape, device=self.device, dtype=dtype))

    # -- one step (lib/gconv_lstm.py:77-221) -----------------------------------------
    def __call__(self, inputs, state, scope=None):
        if self._state_is_tuple:
            c, h = state
        else:
            c, h = torch.split(state, self._nNode, dim=1)  # tf.split(state, 2, axis=1) (:82)
        new_c, new_h = _CellStep.apply(inputs, c, h, self.Wx, self.Wh, self.b, self)
        if self._state_is_tuple:
            new_state = LSTMStateTuple(new_c, new_h)
        else:
            new_state = torch.cat([new_c, new_h], 1)  # tf.concat([new_c, new_h], 1) (:220)
        return new_h, new_state


class _CellStep(torch.autograd.Function):
    """One cell step: x-conv, h-conv (4 gates each, one basis per input),
    fused gates; backward = gates backward, two chebyshev5 backwards, bias sum."""

    @staticmethod
    def forward(ctx, x, c, h, Wx, Wh, b, cell: GConvLSTMCell):
        H, K = cell._num_units, cell._K
        plan = cell.plan
        x, c, h = x.contiguous(), c.contiguous(), h.contiguous()
        basis_x, gx = ops.cheb_forward(plan, x, Wx, K)
        if cell.fused:
            N, M, _ = h.shape
            planes = torch.empty((max(K - 1, 1), N * M, H), device=h.device, dtype=torch.float32)
            c_out, h_out, act = ops.lstm_hconv_step(plan, h, c, gx, Wh, b, K, cell.gates,
                                                    planes=planes[0], plane_stride=N * M * H)
            ctx.save_for_backward(basis_x, planes, h, Wx, Wh, act, c, c_out)
        else:
            basis_h, gh = ops.cheb_forward(plan, h, Wh, K)
            c_out, h_out, act = ops.lstm_cell_forward(gx, gh, b, c, H, cell.gates)
            ctx.save_for_backward(basis_x, basis_h, h, Wx, Wh, act, c, c_out)
        ctx.cell = cell
        return c_out, h_out

    @staticmethod
    def backward(ctx, dc_out, dh_out):
        basis_x, hb, h, Wx, Wh, act, c, c_out = ctx.saved_tensors
        cell = ctx.cell
        H, K, plan = cell._num_units, cell._K, cell.plan
        dh = dh_out.contiguous() if dh_out is not None else None
        dc = dc_out.contiguous() if dc_out is not None else None
        if cell.fused and cell.seq:  # one launch: gates backward + the h-conv's dh
            dpre, dc_prev, dh_prev = ops.lstm_bwd_step(plan, dh, None, dc, act, c, c_out, Wh, K,
                                                       cell.gates)
        else:
            dpre, dc_prev = ops.lstm_cell_backward(dh, None, dc, act, c, c_out, H, cell.gates)
        dx, dWx = ops.cheb_backward(plan, dpre, basis_x, Wx, K, need_dx=ctx.needs_input_grad[0])
        if cell.fused:
            if not cell.seq:
                dh_prev, _ = ops.cheb_backward(plan, dpre, None, Wh, K, need_dW=False)
            dWh = _hweight_grad_planes([h.view(-1, H)], [hb[k] for k in range(K - 1)], [dpre], H, K)
        else:
            dh_prev, dWh = ops.cheb_backward(plan, dpre, hb, Wh, K)
        db = ops.bias_grad(dpre)
        return dx, dc_prev, dh_prev, dWx, dWh, db, None


def _hweight_grad_planes(t0_parts, planes, dpre_parts, H: int, K: int):
    """dWh [K*H, 4H] (row c*K + k) from the Chebyshev orders of h kept as
    planes: order 0 is h itself, given as row blocks t0_parts matched with
    dpre_parts (summed with one cg_weight_grad each, accumulated); order k >= 1
    is planes[k-1] (rows matching the concatenation of dpre_parts)."""
    dev = dpre_parts[0].device
    tmp = torch.empty((K, H, 4 * H), device=dev, dtype=torch.float32)
    for i, (a, d) in enumerate(zip(t0_parts, dpre_parts)):
        ops.weight_grad(a, d, out=tmp[0], accumulate=i > 0)
    dcat = dpre_parts[0] if len(dpre_parts) == 1 else None
    for k in range(1, K):
        if dcat is not None:
            ops.weight_grad(planes[k - 1], dcat, out=tmp[k])
        else:  # the planes' rows follow the concatenation of dpre_parts
            off = 0
            for i, d in enumerate(dpre_parts):
                rows = d.numel() // (4 * H)
                ops.weight_grad(planes[k - 1].reshape(-1, H)[off:off + rows], d, out=tmp[k],
                                accumulate=i > 0)
                off += rows
    return tmp.permute(1, 0, 2).reshape(K * H, 4 * H)


class _Layer(torch.autograd.Function):
    """static_rnn of one cell over a [T, N, M, F] sequence (time-batched x-conv,
    T h-convs, BPTT with one weight-gradient GEMM for the h-weights)."""

    @staticmethod
    def forward(ctx, xs, c0, h0, Wx, Wh, b, cell: GConvLSTMCell, zero_init: bool,
                check_now: bool, want_c: bool = True):
        H, K, plan, gates = cell._num_units, cell._K, cell.plan, cell.gates
        xs = xs.contiguous()
        T, N, M, F = xs.shape
        R = N * M
        dev = xs.device
        f32 = dict(device=dev, dtype=torch.float32)
        seq_x = cell.seq and cell.seq_x
        if seq_x:  # the x-conv inside the sequence kernel; its basis kept as planes
            basis_x, gx = torch.empty((K, T * R, F), device=dev, dtype=torch.float32), None
        else:  # x-conv of every step at once: a batch of T*N samples
            basis_x, gx = ops.cheb_forward(plan, xs.view(T * N, M, F), Wx, K)
            gx = gx.view(T, R, 4 * H)
        hs = torch.empty((T, N, M, H), **f32)
        cs = torch.empty((T, N, M, H), **f32)
        act = torch.empty((T, R, 4 * H), **f32)  # unit-major [R][H][4] on the seq path
        fused = cell.fused or cell.seq
        # h bases kept for the backward's weight gradient: the fused h-step
        # writes the orders 1..K-1 as planes [K-1][T][R][H] (order 0 is h_prev)
        planes = torch.empty((max(K - 1, 1), T, R, H), **f32) if fused and not cell.seq else None
        basis_h = None if fused else torch.empty((T, R, H * K), **f32)
        gh = None if fused else torch.empty((N, M, 4 * H), **f32)
        if cell.seq:
            # a hand-off fault of an earlier launch on this plan not reported yet
            ops.lstm_seq_fault(plan, wait=False)
            # all T steps in one launch.  The h basis of every step as K planes
            # [K][T+1][R][H] of one buffer: plane 0 at t = h_{t-1} (hs IS
            # plane 0 shifted by one step, slot 0 = h0), planes k >= 1 written
            # by the kernel -- so the h-weight gradient is ONE planes-layout
            # GEMM over all orders and steps
            hp = torch.empty((K, T + 1, R, H), **f32)
            if not zero_init:
                hp[0, 0].copy_(h0.reshape(R, H))
            elif seq_x:  # no h-conv at step 0: zero rows for the one-pass weight gradients
                hp[:, 0].zero_()
            hs = hp[0, 1:].view(T, N, M, H)
            planes = hp
            if seq_x:
                ops.lstm_seq_forward_x(plan, xs, Wx, Wh, b, K, gates, h0=None if zero_init else h0,
                                       c0=None if zero_init else c0, out_hs=hs, out_cs=cs,
                                       out_act=act, planes=hp[1] if K > 1 else None,
                                       plane_stride=(T + 1) * R * H, xplanes=basis_x)
            else:
                ops.lstm_seq_forward(plan, gx, Wh, b, K, T, N, gates, h0=None if zero_init else h0,
                                     c0=None if zero_init else c0, out_hs=hs, out_cs=cs,
                                     out_act=act, planes=hp[1] if K > 1 else None,
                                     plane_stride=(T + 1) * R * H)
            # a lost pair hand-off leaves NaN in hs / cs / act: an inference call
            # checks the launch before returning its outputs, a training call
            # before its backward consumes them (one event wait, no device sync)
            if check_now:
                ops.lstm_seq_fault(plan, wait=True)
        for t in range(0 if cell.seq else T):
            h_prev = (None if zero_init else h0) if t == 0 else hs[t - 1]
            c_prev = (None if zero_init else c0) if t == 0 else cs[t - 1]
            if h_prev is not None and fused:  # one launch: h-conv + gates
                ops.lstm_hconv_step(plan, h_prev, c_prev, gx[t], Wh, b, K, gates, out_c=cs[t],
                                    out_h=hs[t], out_act=act[t], planes=planes[0, t],
                                    plane_stride=T * R * H)
                continue
            if h_prev is not None:
                ops.cheb_forward(plan, h_prev, Wh, K, out_basis=basis_h[t], out_y=gh)
            ops.lstm_cell_forward(gx[t], gh if h_prev is not None else None, b, c_prev, H, gates,
                                  out_c=cs[t], out_h=hs[t], out_act=act[t])
        ctx.save_for_backward(basis_x, planes if fused else basis_h, Wx, Wh, act, cs, c0, h0, hs)
        ctx.cell, ctx.zero_init, ctx.shape, ctx.fused = cell, zero_init, (T, N, M, F), fused
        ctx.seq_x = seq_x
        # outputs nobody differentiates reach the backward as None (no zero
        # [T, N, M, H] gradient materialised for a sequence read only at its
        # last step: h_T is an output of its own)
        ctx.set_materialize_grads(False)
        cT = cs[T - 1].clone() if want_c else cs.new_empty(0)  # (a 16 MB copy nobody reads)
        return hs, cT, hs[T - 1].clone()

    @staticmethod
    def backward(ctx, dhs, dcT, dhT):
        basis_x, hb, Wx, Wh, act, cs, c0, h0, hs = ctx.saved_tensors
        cell, zero_init, fused = ctx.cell, ctx.zero_init, ctx.fused
        H, K, plan, gates = cell._num_units, cell._K, cell.plan, cell.gates
        if cell.seq:  # a fault already known raises now; the blocking check runs
            # after the backward is queued (a wait here would idle the GPU while
            # the host queues the backward), before any gradient is returned
            ops.lstm_seq_fault(plan, wait=False)
        T, N, M, F = ctx.shape
        R = N * M
        dev = act.device
        dpre = torch.empty((T, R, 4 * H), device=dev, dtype=torch.float32)
        dhs = dhs.contiguous() if dhs is not None else None
        dc = dcT.contiguous() if dcT is not None else None
        dh_last = None  # the gradient of h_{T-1}: through hs and through h_T
        if dhT is not None:
            dh_last = dhT.contiguous() if dhs is None else dhs[T - 1] + dhT
        elif dhs is not None:
            dh_last = dhs[T - 1]

        def dh_at(t):
            return dh_last if t == T - 1 else (None if dhs is None else dhs[t])

        dh_rec = None
        t_first = 1 if zero_init else 0  # first step whose h-conv ran
        for t in range(T - 1, -1, -1):
            c_prev = (None if zero_init else c0) if t == 0 else cs[t - 1]
            if cell.seq and t < t_first:  # no h-conv at this step: pointwise only, act as stored
                _, dc, _ = ops.lstm_bwd_step(plan, dh_at(t), dh_rec, dc,
                                             act[t], c_prev, cs[t], Wh, K, gates, out_dpre=dpre[t],
                                             act_unit_major=True, need_dh_prev=False)
                dh_rec = None
                continue
            if cell.seq and t >= t_first:
                # one launch: gates backward, dBasis = dpre Wh^T on MFMA and the
                # reverse recurrence over L~^T -> the gradient of h_{t-1}
                _, dc, dh_rec = ops.lstm_bwd_step(plan, dh_at(t), dh_rec,
                                                  dc, act[t], c_prev, cs[t], Wh, K, gates,
                                                  out_dpre=dpre[t], act_unit_major=True)
                continue
            # the sequence kernel's act records are unit-major: gate-major for the
            # pointwise kernel (step 0 of a zero-state layer only)
            act_t = act[t].view(R, H, 4).transpose(1, 2).reshape(R, 4 * H) if cell.seq else act[t]
            dpre_t, dc = ops.lstm_cell_backward(dh_at(t), dh_rec, dc, act_t,
                                                c_prev, cs[t], H, gates, out_dpre=dpre[t])
            if t >= t_first:
                dh_rec, _ = ops.cheb_backward(plan, dpre[t].view(N, M, 4 * H),
                                              None if fused else hb[t].view(R, H * K), Wh, K,
                                              need_dW=False)
            else:
                dh_rec = None
        if ctx.seq_x:
            # dWh, dWx and db in ONE pass over dpre: the h planes of every step
            # (a zero-state layer's step 0 has none: the forward zeroed its slots) and
            # the x planes [K][T*R][F] (dx needs no basis)
            dWh, dWx, db = ops.lstm_weight_grads(hb[0, 0:T].reshape(-1, H), (T + 1) * R * H,
                                                 basis_x[0], T * R * F, K, T * R, dpre)
            dxs = None
            if ctx.needs_input_grad[0]:
                dxs, _ = ops.cheb_backward(plan, dpre.view(T * N, M, 4 * H), None, Wx, K,
                                           need_dW=False)
            dx_out = dxs.view(T, N, M, F) if dxs is not None else None
            if cell.seq:  # raises CGError if the forward's launch lost a pair hand-off
                ops.lstm_seq_fault(plan, wait=True)
            return (dx_out, None if zero_init else dc, None if zero_init else dh_rec, dWx, dWh, db,
                    None, None, None, None)
        if T <= t_first:
            dWh = torch.zeros_like(Wh)
        elif cell.seq:  # one GEMM over the K planes of every step with an h-conv
            dWh = ops.weight_grad_planes(hb[0, t_first:T].reshape(-1, H), (T + 1) * R * H, K,
                                         (T - t_first) * R, dpre[t_first:])
        elif fused:
            t0_parts, dparts = [], []
            if t_first == 0:  # step 0 ran its h-conv on h0
                t0_parts.append(h0.reshape(R, H))
                dparts.append(dpre[0])
            if T > 1:
                t0_parts.append(hs[0:T - 1].reshape(-1, H))
                dparts.append(dpre[1:T])
            dWh = _hweight_grad_planes(t0_parts, [hb[k, t_first:T] for k in range(K - 1)], dparts,
                                       H, K)
        else:
            dWh = ops.weight_grad(hb[t_first:], dpre[t_first:])
        dxs, dWx = ops.cheb_backward(plan, dpre.view(T * N, M, 4 * H), basis_x, Wx, K,
                                     need_dx=ctx.needs_input_grad[0])
        db = ops.bias_grad(dpre)
        dx_out = dxs.view(T, N, M, F) if dxs is not None else None
        dc0 = None if zero_init else dc
        dh0 = None if zero_init else dh_rec
        if cell.seq:  # raises CGError if the forward's launch lost a pair hand-off
            ops.lstm_seq_fault(plan, wait=True)
        return dx_out, dc0, dh0, dWx, dWh, db, None, None, None, None


class DropoutWrapper:
    """tf.nn.rnn_cell.DropoutWrapper(cell, output_keep_prob) as glstm_layer
    wraps every layer's cell (lib/gconv_lstm.py:616, :623): the cell's OUTPUTS
    go through tf.nn.dropout (ops.dropout: a HIP kernel, mask regenerated in the
    backward from a per-call seed), its state passes through untouched.  Like
    the reference graph, it drops whenever it is applied (there is no training
    flag); output_keep_prob = 1 is the identity.  The mask stream is seeded
    from ``seed`` and advances every call (TF's own random stream is not
    reproducible here, only its semantics).  With ``seed=None`` every wrapper
    gets its own stream (torch.initial_seed() mixed with the wrapper's creation
    ordinal), so two same-shaped layers never share masks."""

    def __init__(self, cell: GConvLSTMCell, output_keep_prob: float = 1.0, seed: int | None = None):
        if not 0.0 < float(output_keep_prob) <= 1.0:
            raise ValueError(f"output_keep_prob must be in (0, 1], got {output_keep_prob}")
        self.cell = cell
        self.output_keep_prob = float(output_keep_prob)
        if seed is None:
            seed = (torch.initial_seed() * 0x9E3779B97F4A7C15 + next(_DROPOUT_ORDINAL) * 0xBF58476D1CE4E5B9)
        self._seed = int(seed) & ((1 << 64) - 1)
        self._calls = 0

    def next_seed(self) -> int:
        self._calls += 1
        return (self._seed + 0xD1B54A32D192ED03 * self._calls) & ((1 << 64) - 1)

    def __getattr__(self, name):  # state_size, output_size, zero_state, parameters, ...
        # only reached for names not found normally; 'cell' itself missing means
        # an instance built without __init__ (copy / pickle probing): no recursion
        if name == "cell" or name.startswith("__"):
            raise AttributeError(name)
        return getattr(self.cell, name)

    def __call__(self, inputs, state, scope=None):
        out, new_state = self.cell(inputs, state, scope)
        return ops.dropout(out, self.output_keep_prob, self.next_seed()), new_state


def layer(cell, xs: torch.Tensor, initial_state=None, final_c: bool = True):
    """Run ``cell`` over xs [T, N, M, feat_in]; returns (hs [T, N, M, H],
    LSTMStateTuple(c_T, h_T)).  initial_state None = zero state; final_c False
    = the caller does not read c_T (an empty tensor in its place, no copy).

    On the one-launch path a lost pair hand-off (cg_lstm_seq_fault) raises
    CGError: here when no gradient will be taken (the outputs go straight to
    the caller), else in the backward, before any gradient is returned (the
    outputs then hold NaN from the lost step on).

    ``cell`` may be a DropoutWrapper: the returned outputs are then dropped
    out, the state (c_T, h_T) is not (DropoutWrapper semantics)."""
    if isinstance(cell, DropoutWrapper):
        hs, state = layer(cell.cell, xs, initial_state, final_c)
        return ops.dropout(hs, cell.output_keep_prob, cell.next_seed()), state
    ins = [xs, cell.Wx, cell.Wh, cell.b] + ([] if initial_state is None else list(initial_state))
    check_now = not (torch.is_grad_enabled() and any(t.requires_grad for t in ins))
    if initial_state is None:
        z = xs.new_empty(0)  # placeholders: a zero state is never read (no fill launch)
        hs, cT, hT = _Layer.apply(xs, z, z, cell.Wx, cell.Wh, cell.b, cell, True, check_now,
                                  final_c)
    else:
        c0, h0 = initial_state
        hs, cT, hT = _Layer.apply(xs, c0.contiguous(), h0.contiguous(), cell.Wx, cell.Wh, cell.b,
                                  cell, False, check_now, final_c)
    return hs, LSTMStateTuple(cT, hT)


def static_rnn(cells, inputs, initial_states=None):
    """``tf.nn.static_rnn(MultiRNNCell(cells), inputs)`` (lib/gconv_lstm.py:625-626).

    inputs: a list of T tensors [N, M, F] or one [T, N, M, F] tensor.
    Returns (outputs: list of T tensors [N, M, H] of the last layer,
    states: tuple of LSTMStateTuple per layer).  Layer-by-layer evaluation
    equals the reference's time-major one (layer l at step t depends only on
    layer l-1 at step t and layer l at step t-1)."""
    if isinstance(cells, (GConvLSTMCell, DropoutWrapper)):
        cells = [cells]
    xs = torch.stack(list(inputs)) if isinstance(inputs, (list, tuple)) else inputs
    states = []
    for li, cell in enumerate(cells):
        init = None if initial_states is None else initial_states[li]
        xs, st = layer(cell, xs, init)
        states.append(st)
    return list(xs.unbind(0)), tuple(states)


def clip_gradients(params, max_grad_norm, check_numerics: bool = True):
    """gconvRNN.Model._build_optim's gradient clipping (lib/gconvRNN.py:392-402)
    on the parameters' .grad: per variable tf.clip_by_norm(grad, max_grad_norm)
    then tf.check_numerics (raises FloatingPointError on NaN / Inf), in place
    on the HIP kernels.  max_grad_norm None = no clipping (the reference's else
    branch)."""
    if max_grad_norm is None:
        return
    grads = [p.grad for p in params if p.grad is not None]
    ops.clip_by_norm_(grads, float(max_grad_norm), check_numerics)


def unstack_time(x: torch.Tensor, T: int) -> torch.Tensor:
    """inference_glstm's split (lib/gconv_lstm.py:272-275): [N, M, F*T] ->
    reshape [N, M, F, T] -> unstack axis 3 -> [T, N, M, F] (contiguous)."""
    N, M, C = x.shape
    return x.reshape(N, M, C // T, T).permute(3, 0, 1, 2).contiguous()


def dropout_seed(seed: int, rank: int, layer: int) -> int:
    """A 64-bit mask-stream seed from (model seed, rank, layer index): a
    splitmix64 finaliser over the three (deterministic across processes, unlike
    Python's salted ``hash``)."""
    z = (int(seed) * 0x9E3779B97F4A7C15 + int(rank) * 0xBF58476D1CE4E5B9 +
         (int(layer) + 1) * 0x94D049BB133111EB) & ((1 << 64) - 1)
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & ((1 << 64) - 1)
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & ((1 << 64) - 1)
    return z ^ (z >> 31)


class GLSTMModel:
    """``GconvModel.inference_glstm`` (lib/gconv_lstm.py:271-281) trained as
    ``GraphModel`` trains it (lib/graph_model.py:246-310):

      x [N, M, F*T]  --unstack time (:272-275)-->  T x [N, M, F]
      glstm_layer    layer_count GConvLSTMCells under static_rnn (:609-627),
                     each in a DropoutWrapper(output_keep_prob) (:616, :623)
      fc_layer       out = cheby_conv(outputs[-1]; W_fc [K*H, Fout]) (:629-636)
      loss           mean((labels - out)^2) + its moving average    cg_mse_loss_ema
      exchange       ONE all-reduce(sum) of the flat gradient bucket (N > 1)
      update         ONE optimizer launch over the flat parameter buffer,
                     grad_scale = 1/world: Adam (graph_model.py:293, staircase
                     exponential decay) or gconvRNN's sgd / rmsprop
                     (lib/gconvRNN.py:381-389)

    Every parameter (each layer's Wx [K*Fin, 4H], Wh [K*H, 4H], b [4H], then
    W_fc) is a view into one flat fp32 buffer and its ``.grad`` a view into one
    flat gradient bucket that autograd accumulates into in place -- at config E
    (Fin 2, H 32, K 3, one layer) 13 376 floats = 53.5 KB -- so the data-parallel
    exchange of a step is one collective and the update one launch.
    ``comm`` is any object with ``allreduce_sum_(tensor, stream)`` and ``world``
    (``dist.RcclComm`` on RCCL, ``dist.TorchComm`` on a process group)."""

    OPTIMIZERS = ("adam", "sgd", "rmsprop")

    def __init__(self, L, N: int, T: int, feat_in: int, num_hidden: int = 32, K: int = 3,
                 layer_count: int = 1, out_features: int = 2, keep_prob: float = 0.8,
                 optimizer: str = "adam", learning_rate: float = 1e-3, decay_rate: float = 0.95,
                 decay_steps: int | None = None, lmax: float = 2, gates: str = "reference",
                 device=None, seed: int = 2017, comm=None):
        if optimizer not in self.OPTIMIZERS:
            raise ValueError(f"optimizer must be one of {self.OPTIMIZERS}")
        self.device = torch.device(device if device is not None else "cuda")
        self.N, self.T, self.F, self.H, self.K = int(N), int(T), int(feat_in), int(num_hidden), int(K)
        self.Fout = int(out_features)
        self.optimizer, self.lr = optimizer, learning_rate
        self.decay_rate, self.decay_steps = decay_rate, decay_steps
        self.comm = comm
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed)
        cells = []
        for li in range(int(layer_count)):
            fin = self.F if li == 0 else self.H
            cells.append(GConvLSTMCell(self.H, laplacian=L, lmax=lmax, K=self.K, feat_in=fin,
                                       gates=gates, device=self.device, generator=gen))
        self.plan = cells[0].plan
        self.M = self.plan.M
        H, K = self.H, self.K
        sizes = [c.Wx.numel() + c.Wh.numel() + c.b.numel() for c in cells] + [K * H * self.Fout]
        f32 = dict(device=self.device, dtype=torch.float32)
        total = sum(sizes)
        self.flat = torch.empty(total, **f32)
        self.grad = torch.zeros(total, **f32)
        self.names, self.params = [], []
        off = 0

        def bind(t_init, name):
            nonlocal off
            n = t_init.numel()
            view = self.flat[off:off + n].view_as(t_init)
            view.copy_(t_init)
            p = torch.nn.Parameter(view)   # aliases the flat buffer
            p.grad = self.grad[off:off + n].view_as(t_init)
            off += n
            self.names.append(name)
            self.params.append(p)
            return p

        scope = "gconv_lstm_layer/rnn/multi_rnn_cell/cell_{}/"
        for li, c in enumerate(cells):
            with torch.no_grad():
                c.Wx = bind(c.Wx.detach(), scope.format(li) + "Wx")
                c.Wh = bind(c.Wh.detach(), scope.format(li) + "Wh")
                c.b = bind(c.b.detach(), scope.format(li) + "b")
        with torch.no_grad():
            w0 = truncated_normal_(torch.empty((K * H, self.Fout), **f32), 0.1, gen)
            self.W_fc = bind(w0, "conv_init/weights")
        assert off == total
        self.cells = cells
        # each wrapper's mask stream from (model seed, rank, layer): training is
        # reproducible from the seed, and the ranks draw independent masks for
        # their shards (TF: one random op per wrapper per replica)
        rank = int(getattr(comm, "rank", 0)) if comm is not None else 0
        self.wrapped = [DropoutWrapper(c, keep_prob, seed=dropout_seed(seed, rank, li))
                        if keep_prob < 1.0 else c for li, c in enumerate(cells)]
        # optimizer slots (TF 1.x: Adam m, v zeros; RMSProp ms ONES, mom zeros)
        self.s1 = (torch.ones if optimizer == "rmsprop" else torch.zeros)(total, **f32)
        self.s2 = torch.zeros(total, **f32)
        self.loss = torch.empty((1,), **f32)
        self.ema = torch.zeros((3,), **f32)  # ExponentialMovingAverage(0.9) of the loss
        self.dout = torch.empty((self.N, self.M, self.Fout), **f32)
        nb = ctypes.c_size_t()
        _lib.call("cg_mse_loss_workspace_bytes", self.N * self.M * self.Fout, ctypes.byref(nb))
        self.mws = torch.empty(max(nb.value, 1), device=self.device, dtype=torch.uint8)
        self.mws_n = nb.value
        self.step_count = 0

    @property
    def world(self):
        return self.comm.world if self.comm is not None else 1

    @property
    def loss_average(self):
        return self.ema[1:2]

    def parameters(self):
        return dict(zip(self.names, self.params))

    def gradients(self):
        return dict(zip(self.names, (p.grad for p in self.params)))

    def learning_rate(self, step):
        """tf.train.exponential_decay(lr, global_step, decay_steps, decay_rate, staircase=True)."""
        if self.decay_rate == 1 or not self.decay_steps:
            return self.lr
        return self.lr * self.decay_rate ** math.floor(step / self.decay_steps)

    def _steps(self, x):
        if x.dim() == 3:  # [N, M, F*T] as the reference feeds it
            return unstack_time(x, self.T)
        return x.contiguous()

    def forward(self, x):
        """inference_glstm: the fc layer's output [N, M, out_features].

        static_rnn(self.wrapped, ...) then outputs[-1], with the last layer's
        sequence read at its last step only: that layer runs unwrapped, its
        h_T (a separate output: the backward gets no zero [T, N, M, H]
        gradient) goes through the dropout as the last-step slice of the
        layer's mask (same seed, element offset (T-1)*N*M*H) -- the values
        and gradients of the whole-sequence form, 1/T of its dropout traffic."""
        xs = self._steps(x)
        last = len(self.wrapped) - 1
        for li, cell in enumerate(self.wrapped):
            if li < last:
                xs, _ = layer(cell, xs, final_c=False)
                continue
            drop = isinstance(cell, DropoutWrapper)
            _, st = layer(cell.cell if drop else cell, xs, final_c=False)
            h = st.h
            if drop:
                h = ops.dropout(h, cell.output_keep_prob, cell.next_seed(),
                                offset=(xs.shape[0] - 1) * h.numel())
        return ops.cheb_conv(h, self.W_fc, self.plan, self.K)

    def train_step(self, x, labels, stream=None):
        """One optimizer step; returns the device loss [1] (this rank's batch)."""
        s = stream if stream is not None else torch.cuda.current_stream(self.device).cuda_stream
        self.grad.zero_()
        out = self.forward(x)
        labels = labels.contiguous()
        if labels.numel() != out.numel():
            raise ValueError("labels must match the logits' shape")
        _lib.call("cg_mse_loss_ema", out.data_ptr(), labels.data_ptr(), out.numel(),
                  self.loss.data_ptr(), self.dout.data_ptr(), self.ema.data_ptr(),
                  ctypes.c_float(0.9), self.mws.data_ptr(), self.mws_n, s)
        out.backward(self.dout)
        for p in self.params:  # autograd accumulated into the flat bucket in place
            if p.grad is None or p.grad.data_ptr() < self.grad.data_ptr() or \
                    p.grad.data_ptr() >= self.grad.data_ptr() + 4 * self.grad.numel():
                raise RuntimeError("a parameter's .grad left the flat gradient bucket")
        world = 1
        if self.comm is not None and self.comm.world > 1:
            self.comm.allreduce_sum_(self.grad, s)
            world = self.comm.world
        self.step_count += 1
        lr = self.learning_rate(self.step_count - 1)
        n = self.flat.numel()
        if self.optimizer == "adam":
            _lib.call("cg_adam_update", self.flat.data_ptr(), self.grad.data_ptr(), self.s1.data_ptr(),
                      self.s2.data_ptr(), n, ctypes.c_float(lr), ctypes.c_float(0.9),
                      ctypes.c_float(0.999), ctypes.c_float(1e-8), self.step_count,
                      ctypes.c_float(1.0 / world), s)
        elif self.optimizer == "sgd":
            _lib.call("cg_sgd_update", self.flat.data_ptr(), self.grad.data_ptr(), n,
                      ctypes.c_float(lr), ctypes.c_float(1.0 / world), s)
        else:
            _lib.call("cg_rmsprop_update", self.flat.data_ptr(), self.grad.data_ptr(),
                      self.s1.data_ptr(), self.s2.data_ptr(), n, ctypes.c_float(lr),
                      ctypes.c_float(0.9), ctypes.c_float(0.0), ctypes.c_float(1e-10),
                      ctypes.c_float(1.0 / world), s)
        return self.loss
