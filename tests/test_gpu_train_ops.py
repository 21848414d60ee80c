"""Training-loop pieces of the gconv-LSTM models on the HIP kernels:
DropoutWrapper(output_keep_prob) of glstm_layer (lib/gconv_lstm.py:616, :623;
tf.nn.dropout 1.x: y = (x / keep) * floor(keep + u)) and gconvRNN.Model's
tf.clip_by_norm + tf.check_numerics (lib/gconvRNN.py:392-402).  TF's random
stream is not reproducible here: the dropout tests pin the formula, the mask's
regeneration in the backward and the keep rate, not TF's draws."""
import math

import numpy as np
import pytest
import scipy.sparse

from conftest import case, load_golden
from oracle import cheb_oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev(built_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cnn_graph_amd import _lib
    _lib.lib()
    return torch.device("cuda", 0)


def test_dropout_formula_mask_and_rate(dev):
    from cnn_graph_amd import ops
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    n, keep = 1 << 20, 0.8
    x = torch.randn((n,), device=dev, generator=g)
    xa = x.clone().requires_grad_()
    y = ops.dropout(xa, keep, seed=1234)
    dy = torch.randn((n,), device=dev, generator=g)
    y.backward(dy)
    torch.cuda.synchronize()
    # the mask itself, from dropping a tensor of ones with the same seed (y != 0
    # would misread a kept exact zero of x)
    mask = ops.dropout(torch.ones_like(x), keep, seed=1234) != 0
    kept = int(mask.sum())
    # binomial(n, 0.8): 6 sigma
    assert abs(kept - keep * n) < 6 * math.sqrt(n * keep * (1 - keep))
    # IEEE fp32 division on the host (torch divides a GPU tensor by a CPU scalar
    # as a multiply by its reciprocal, which is not the formula)
    k32 = np.float32(keep)
    xn, yn, mn = x.cpu().numpy(), y.detach().cpu().numpy(), mask.cpu().numpy()
    mf = mn.astype(np.float32)
    assert np.array_equal(yn, (xn / k32) * mf)
    dyn = dy.cpu().numpy()
    gn = xa.grad.cpu().numpy()
    ref = (dyn * mf) / k32
    bad = np.flatnonzero(gn != ref)
    info = [(int(i), float(dyn[i]), bool(mn[i]), float(gn[i]), float(ref[i])) for i in bad[:5]]
    assert bad.size == 0, (bad.size, info)
    # deterministic in the seed, another seed another mask
    assert torch.equal(ops.dropout(x, keep, 1234), y.detach())
    assert not torch.equal(ops.dropout(torch.ones_like(x), keep, 1235) != 0, mask)
    assert ops.dropout(x, 1.0, 7) is x


def test_dropout_wrapper_layer_outputs_only(dev):
    """DropoutWrapper: outputs dropped, state (c_T, h_T) not; a 2-layer
    static_rnn feeds the dropped outputs to the next layer."""
    from cnn_graph_amd import ops
    from cnn_graph_amd.gconv_lstm import DropoutWrapper, GConvLSTMCell, layer, static_rnn
    c = case(load_golden("golden_E.npz"))
    M = c["M"]
    Lt = scipy.sparse.csr_matrix((c["Lt_val"], c["Lt_col"], c["Lt_rowptr"]), shape=(M, M))
    L = (Lt + scipy.sparse.identity(M, dtype=np.float32, format="csr")).tocsr()
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    cell = GConvLSTMCell(32, laplacian=L, lmax=2, K=3, feat_in=2, device=dev, generator=g)
    xs = torch.rand((4, 2, M, 2), device=dev, generator=g)
    with torch.no_grad():
        hs, (cT, hT) = layer(cell, xs)
        w = DropoutWrapper(cell, 0.8, seed=99)
        hd, (cT2, hT2) = layer(w, xs)
        ref = ops.dropout(hs, 0.8, DropoutWrapper(cell, 0.8, seed=99).next_seed())
    assert torch.equal(hd, ref)
    assert torch.equal(cT2, cT) and torch.equal(hT2, hT) and torch.equal(hT2, hs[-1])
    cell2 = GConvLSTMCell(32, laplacian=L, lmax=2, K=3, feat_in=32, device=dev, generator=g)
    w1, w2 = DropoutWrapper(cell, 0.8, seed=5), DropoutWrapper(cell2, 0.8, seed=6)
    with torch.no_grad():
        outs, states = static_rnn([w1, w2], xs)
        h1, _ = layer(cell, xs)
        d1 = ops.dropout(h1, 0.8, DropoutWrapper(cell, 0.8, seed=5).next_seed())
        h2, _ = layer(cell2, d1)
        d2 = ops.dropout(h2, 0.8, DropoutWrapper(cell2, 0.8, seed=6).next_seed())
    assert torch.equal(torch.stack(outs), d2)
    assert torch.equal(states[1].h, h2[-1])


def test_dropout_mask_matches_host_restatement(dev):
    """The kernel's mask is floor(keep + u) with u the host restatement of the
    draw (tests/test_dropout_cpu.py), element for element, both kernels."""
    from cnn_graph_amd import ops
    from test_dropout_cpu import draws
    n, keep, seed = 50001, 0.8, 0x0123456789ABCDEF
    u = draws(seed, n)
    ref = np.floor(np.float32(keep) + u)
    ones = torch.ones((n + 1,), device=dev)
    got4 = (ops.dropout(ones[:n], keep, seed) != 0).cpu().numpy()  # aligned: k_dropout4
    got1 = (ops.dropout(ones[1:], keep, seed) != 0).cpu().numpy()  # misaligned: k_dropout
    assert np.array_equal(got4, ref != 0)
    assert np.array_equal(got1, ref != 0)


def test_dropout_vector_and_offset_slices(dev):
    """The four-per-thread kernel (16-byte aligned x / y) and the scalar one
    (misaligned) draw the same bits; a slice dropped with offset = its first
    element's index equals that slice of the whole tensor's dropout, forward
    and backward (GLSTMModel drops only the last step of its last layer this
    way)."""
    from cnn_graph_amd import ops
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    n, keep, seed = 100003, 0.8, 0xFEEDFACECAFEBEEF
    x = torch.randn((n,), device=dev, generator=g)
    y = ops.dropout(x, keep, seed)
    buf = torch.empty((n + 1,), device=dev)
    buf[1:].copy_(x)  # 4-byte offset: the scalar kernel
    assert torch.equal(ops.dropout(buf[1:], keep, seed), y)
    for off, m in ((0, 7), (4, 4096), (13, 1001), (n - 5, 5), (64 * 1024, 30000)):
        xs = x[off:off + m].clone().requires_grad_()
        ys = ops.dropout(xs, keep, seed, offset=off)
        assert torch.equal(ys, y[off:off + m]), off
        dy = torch.randn((m,), device=dev, generator=g)
        ys.backward(dy)
        full = x.clone().requires_grad_()
        dfull = torch.zeros((n,), device=dev)
        dfull[off:off + m] = dy
        ops.dropout(full, keep, seed).backward(dfull)
        assert torch.equal(xs.grad, full.grad[off:off + m]), off


def test_glstm_forward_last_step_equals_static_rnn(dev):
    """GLSTMModel.forward reads the last layer at its last step only (h_T as
    its own output, the dropout on that slice with the mask offset): output
    and every gradient equal the whole-sequence form static_rnn(wrapped) +
    outputs[-1] (lib/gconv_lstm.py:625-636), bitwise, for 1 and 2 layers."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__)))
    import glstm_dp_worker as Wk
    from cnn_graph_amd import ops
    from cnn_graph_amd.gconv_lstm import GLSTMModel, static_rnn
    L, x, labels = Wk.problem()
    xs = torch.from_numpy(x[:2]).to(dev)
    for layers in (1, 2):
        ms = [GLSTMModel(L, 2, Wk.T, Wk.FIN, num_hidden=Wk.H, K=Wk.K, out_features=Wk.FOUT,
                         layer_count=layers, keep_prob=0.8, device=dev, seed=21) for _ in range(2)]
        a, b = ms
        ya = a.forward(xs)
        outs, _ = static_rnn(b.wrapped, b._steps(xs))
        yb = ops.cheb_conv(outs[-1].contiguous(), b.W_fc, b.plan, b.K)
        assert torch.equal(ya, yb), layers
        dy = torch.randn(ya.shape, device=dev, generator=torch.Generator(device=dev).manual_seed(5))
        a.grad.zero_()
        b.grad.zero_()
        ya.backward(dy)
        yb.backward(dy)
        torch.cuda.synchronize()
        assert a.grad.abs().sum() > 0
        assert torch.equal(a.grad, b.grad), (layers, float((a.grad - b.grad).abs().max()))


def test_clip_by_norm_and_check_numerics(dev):
    from cnn_graph_amd import ops
    rng = np.random.default_rng(4)
    a = rng.standard_normal(5000).astype(np.float32) * 3
    b = rng.standard_normal((96, 128)).astype(np.float32) * 1e-3
    ta, tb = torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev)
    ops.clip_by_norm_([ta, tb], 5.0)
    torch.cuda.synchronize()
    for t, ref in ((ta, a), (tb, b)):
        r64 = ref.astype(np.float64)
        nrm = np.sqrt((r64 * r64).sum())
        assert O.normwise_err(t.cpu().numpy(), r64 * 5.0 / max(nrm, 5.0)) < 1e-6
    # norm < 5: t = (t*5)/max(norm, 5) = (t*5)/5 in IEEE fp32 (numpy divides
    # correctly rounded; torch's tensor / scalar multiplies by the reciprocal)
    f5 = np.float32(5.0)
    assert np.array_equal(tb.cpu().numpy(), (b * f5) / f5)
    bad = torch.ones((100,), device=dev)
    bad[17] = float("nan")
    with pytest.raises(FloatingPointError):
        ops.clip_by_norm_([ta, bad], 5.0)
    ok = torch.ones((100,), device=dev)
    ok[3] = float("inf")
    ops.clip_by_norm_([ok], 5.0, check_numerics=False)  # no check: no raise
