"""gconv-LSTM cell (lib/gconv_lstm.py:77-221) on the HIP path vs the float64
oracle (oracle/lstm_oracle.py).  Bar: max-abs-normalised error <= 1e-5
(the north star's 1e-5 rel-fp32), on forward states and every gradient."""
import numpy as np
import pytest
import scipy.sparse

from conftest import case, load_golden
from oracle import cheb_oracle as O
from oracle import lstm_oracle as LO

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

TOL = 1e-5


@pytest.fixture(scope="module")
def dev(built_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cnn_graph_amd import _lib
    _lib.lib()
    return torch.device("cuda", 0)


def t(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(dev)


def graph_E(name="E"):
    """config E's grid graph (or another config's golden graph by name);
    returns (L~ scipy, lap tuple for the oracle, M)."""
    c = case(load_golden(f"golden_{name}.npz"))
    M = c["M"]
    Lt = scipy.sparse.csr_matrix((c["Lt_val"], c["Lt_col"], c["Lt_rowptr"]), shape=(M, M))
    return Lt, (c["Lt_rowptr"], c["Lt_col"], c["Lt_val"].astype(np.float64)), M


def make_cell(Lt, feat_in, H, K, gates, dev, seed, hconv="auto"):
    """A cell on L~ directly (lmax=2 rescale happens in plan_for, so hand it
    the plan of L~ by constructing from L = L~ + I: rescale_L(L, 2) = L~)."""
    from cnn_graph_amd.gconv_lstm import GConvLSTMCell
    L = (Lt + scipy.sparse.identity(Lt.shape[0], dtype=np.float32, format="csr")).tocsr()
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    cell = GConvLSTMCell(H, laplacian=L, lmax=2, K=K, feat_in=feat_in, gates=gates, device=dev,
                         generator=g, hconv=hconv)
    return cell, L


def params_np(cell):
    return [cell.Wx.detach().cpu().numpy().astype(np.float64),
            cell.Wh.detach().cpu().numpy().astype(np.float64),
            cell.b.detach().cpu().numpy().astype(np.float64)]


def oracle_lap(cell, L):
    """The L~ the plan actually holds (rescale_L of the cell's L)."""
    rp, ci, v = cell.plan.rowptr, cell.plan.col, cell.plan.val
    return (rp, ci, v.astype(np.float64))


@pytest.mark.parametrize("gates", ["reference", "standard"])
def test_pointwise_cell_kernels_vs_numpy(dev, gates):
    from cnn_graph_amd import ops
    rng = np.random.default_rng(3)
    R, H = 1000, 24
    gx = rng.standard_normal((R, 4 * H)) * 0.5
    gh = rng.standard_normal((R, 4 * H)) * 0.5
    b = rng.standard_normal(4 * H) * 0.2
    c = rng.standard_normal((R, H))
    dh, dh2, dc = (rng.standard_normal((R, H)) for _ in range(3))
    gx32, gh32, b32, c32 = (a.astype(np.float32).astype(np.float64) for a in (gx, gh, b, c))
    c_out, h_out, act = ops.lstm_cell_forward(t(gx, dev), t(gh, dev), t(b, dev), t(c, dev), H, gates)
    dpre, dcp = ops.lstm_cell_backward(t(dh, dev), t(dh2, dev), t(dc, dev), act, t(c, dev), c_out, H,
                                       gates)
    torch.cuda.synchronize()
    # the kernel's inputs are fp32 and so is its pre-activation sum; tan / tanh
    # / sigmoid and everything after are checked against float64 from there
    a = ((gx.astype(np.float32) + gh.astype(np.float32)) + b.astype(np.float32)).astype(np.float64)
    sig = lambda v: 1 / (1 + np.exp(-v))  # noqa: E731
    z = np.tan(a[:, :H]) if gates == "reference" else np.tanh(a[:, :H])
    i, f = sig(a[:, H:2 * H]), sig(a[:, 2 * H:3 * H])
    o = np.tanh(a[:, 3 * H:]) if gates == "reference" else sig(a[:, 3 * H:])
    cn = f * c32 + i * z
    hn = o * np.tanh(cn)
    assert O.normwise_err(c_out.cpu().numpy(), cn) < TOL
    assert O.normwise_err(h_out.cpu().numpy(), hn) < TOL
    assert O.normwise_err(act.cpu().numpy(), np.concatenate([z, i, f, o], 1)) < TOL
    dh_t = dh.astype(np.float32).astype(np.float64) + dh2.astype(np.float32).astype(np.float64)
    tc = np.tanh(cn)
    dcn = dh_t * o * (1 - tc ** 2) + dc.astype(np.float32)
    d_o = dh_t * tc
    daz = dcn * i * ((1 + z * z) if gates == "reference" else (1 - z * z))
    dao = d_o * ((1 - o * o) if gates == "reference" else o * (1 - o))
    ref = np.concatenate([daz, dcn * z * i * (1 - i), dcn * c32 * f * (1 - f), dao], 1)
    assert O.normwise_err(dpre.cpu().numpy(), ref) < TOL
    assert O.normwise_err(dcp.cpu().numpy(), dcn * f) < TOL


def test_weight_and_bias_grad_accumulate(dev):
    from cnn_graph_amd import ops
    rng = np.random.default_rng(5)
    R, FK, Fo = 70000, 96, 128
    A = rng.standard_normal((R, FK)).astype(np.float32)
    D = rng.standard_normal((R, Fo)).astype(np.float32)
    W0 = rng.standard_normal((FK, Fo)).astype(np.float32)
    out = t(W0, dev)
    ops.weight_grad(t(A, dev), t(D, dev), out=out, accumulate=True)
    db = ops.bias_grad(t(D, dev))
    torch.cuda.synchronize()
    ref = W0.astype(np.float64) + A.astype(np.float64).T @ D.astype(np.float64)
    assert O.normwise_err(out.cpu().numpy(), ref) < TOL
    assert O.normwise_err(db.cpu().numpy(), D.astype(np.float64).sum(0)) < TOL
    # bitwise reproducible (fixed-order reductions)
    again = ops.weight_grad(t(A, dev), t(D, dev))
    again2 = ops.weight_grad(t(A, dev), t(D, dev))
    assert torch.equal(again, again2)


@pytest.mark.parametrize("gates", ["reference", "standard"])
@pytest.mark.parametrize("H,K", [(8, 3), (32, 3), (32, 2), (32, 4)])
def test_cell_step_autograd_vs_oracle(dev, gates, H, K):
    """GConvLSTMCell.__call__ with a non-zero state, gradients by autograd
    (H = 32: the one-launch h-step, cg_lstm_hconv_step)."""
    Lt, _, M = graph_E()
    N, Fin = 3, 2
    cell, L = make_cell(Lt, Fin, H, K, gates, dev, seed=11)
    assert cell.fused == (H == 32)
    lap = oracle_lap(cell, L)
    rng = np.random.default_rng(2)
    x, c0, h0 = rng.standard_normal((N, M, Fin)), rng.standard_normal((N, M, H)) * 0.5, \
        rng.standard_normal((N, M, H)) * 0.5
    gh, gc = rng.standard_normal((N, M, H)), rng.standard_normal((N, M, H))
    xt, ct, ht = (t(a, dev).requires_grad_() for a in (x, c0, h0))
    new_h, (new_c, new_h2) = cell(xt, (ct, ht))
    assert new_h2 is new_h
    loss = (new_h * t(gh, dev)).sum() + (new_c * t(gc, dev)).sum()
    loss.backward()
    torch.cuda.synchronize()
    p = params_np(cell)
    f32 = lambda a: a.astype(np.float32).astype(np.float64)  # noqa: E731
    cn, hn, cache = LO.cell_forward(f32(x), f32(c0), f32(h0), *p, lap, K, H, gates)
    dx, dc, dh, dWx, dWh, db, _ = LO.cell_backward(f32(gh), f32(gc), cache, p[0], p[1], lap, K, H, gates)
    assert O.normwise_err(new_c.detach().cpu().numpy(), cn) < TOL
    assert O.normwise_err(new_h.detach().cpu().numpy(), hn) < TOL
    for name, got, ref in (("dx", xt.grad, dx), ("dc", ct.grad, dc), ("dh", ht.grad, dh),
                           ("dWx", cell.Wx.grad, dWx), ("dWh", cell.Wh.grad, dWh), ("db", cell.b.grad, db)):
        err = O.normwise_err(got.cpu().numpy(), ref)
        assert err < TOL, (name, err)


@pytest.mark.parametrize("zero_init", [True, False])
@pytest.mark.parametrize("H", [8, 32])
def test_two_layer_static_rnn_vs_oracle(dev, zero_init, H):
    """static_rnn(MultiRNNCell([cell1, cell2])) (lib/gconv_lstm.py:609-627),
    T=4, zero or given initial state, full BPTT (H = 32: fused h-steps)."""
    from cnn_graph_amd.gconv_lstm import static_rnn
    Lt, _, M = graph_E()
    T, N, Fin, K = 4, 2, 2, 3
    cell1, L = make_cell(Lt, Fin, H, K, "reference", dev, seed=21)
    cell2, _ = make_cell(Lt, H, H, K, "reference", dev, seed=22)
    lap = oracle_lap(cell1, L)
    rng = np.random.default_rng(4)
    xs = rng.standard_normal((T, N, M, Fin))
    gh = rng.standard_normal((T, N, M, H))
    init = None
    inits_np = [(None, None), (None, None)]
    if not zero_init:
        st = [rng.standard_normal((N, M, H)) * 0.5 for _ in range(4)]
        inits_np = [(st[0], st[1]), (st[2], st[3])]
        init = [tuple(t(a, dev).requires_grad_() for a in pair) for pair in inits_np]
    xt = t(xs, dev).requires_grad_()
    outs, states = static_rnn([cell1, cell2], list(xt.unbind(0)), init)
    loss = (torch.stack(outs) * t(gh, dev)).sum()
    loss.backward()
    torch.cuda.synchronize()
    f32 = lambda a: None if a is None else a.astype(np.float32).astype(np.float64)  # noqa: E731
    p1, p2 = params_np(cell1), params_np(cell2)
    h1, c1, ca1 = LO.layer_forward(f32(xs), p1, lap, K, H, f32(inits_np[0][0]), f32(inits_np[0][1]))
    h2, c2, ca2 = LO.layer_forward(h1, p2, lap, K, H, f32(inits_np[1][0]), f32(inits_np[1][1]))
    assert O.normwise_err(torch.stack(outs).detach().cpu().numpy(), h2) < TOL
    assert O.normwise_err(states[0].c.detach().cpu().numpy(), c1[-1]) < TOL
    dh1, dc02, dh02, dWx2, dWh2, db2 = LO.layer_backward(f32(gh), None, ca2, p2, lap, K, H)
    dxs, dc01, dh01, dWx1, dWh1, db1 = LO.layer_backward(dh1, None, ca1, p1, lap, K, H)
    pairs = [("dxs", xt.grad, dxs), ("dWx1", cell1.Wx.grad, dWx1), ("dWh1", cell1.Wh.grad, dWh1),
             ("db1", cell1.b.grad, db1), ("dWx2", cell2.Wx.grad, dWx2), ("dWh2", cell2.Wh.grad, dWh2),
             ("db2", cell2.b.grad, db2)]
    if not zero_init:
        pairs += [("dc0_1", init[0][0].grad, dc01), ("dh0_1", init[0][1].grad, dh01),
                  ("dc0_2", init[1][0].grad, dc02), ("dh0_2", init[1][1].grad, dh02)]
    for name, got, ref in pairs:
        err = O.normwise_err(got.cpu().numpy(), ref)
        assert err < TOL, (name, err)


def test_config_E_sequence_path_equals_cell_steps(dev):
    """Config E at full size (M=1024, T=12, K=3, Fin=2, H=32, N=128): the fused
    sequence path (time-batched x-conv, one dW GEMM for Wh) equals stepping the
    cell T times under autograd (a size-independent identity), and a small
    batch of it matches the oracle."""
    from cnn_graph_amd.gconv_lstm import layer
    Lt, _, M = graph_E()
    T, N, Fin, H, K = 12, 128, 2, 32, 3
    cell, L = make_cell(Lt, Fin, H, K, "reference", dev, seed=31)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    xs = torch.randn((T, N, M, Fin), device=dev, generator=g)
    gh = torch.randn((T, N, M, H), device=dev, generator=g)
    xa = xs.clone().requires_grad_()
    hs, _ = layer(cell, xa)
    (hs * gh).sum().backward()
    ga = [p.grad.clone() for p in cell.parameters()] + [xa.grad.clone()]
    for p in cell.parameters():
        p.grad = None
    xb = xs.clone().requires_grad_()
    c, h = cell.zero_state(N)
    outs = []
    for s in range(T):
        h, (c, _) = cell(xb[s], (c, h))
        outs.append(h)
    hb = torch.stack(outs)
    (hb * gh).sum().backward()
    gb = [p.grad for p in cell.parameters()] + [xb.grad]
    torch.cuda.synchronize()
    assert O.normwise_err(hs.detach().cpu().numpy(), hb.detach().cpu().numpy()) < 1e-6
    for a, b in zip(ga, gb):
        assert O.normwise_err(a.cpu().numpy(), b.cpu().numpy()) < 1e-5
    # oracle on the first 4 samples (the filter is per-sample independent)
    lap = oracle_lap(cell, L)
    n = 4
    f64 = lambda a: a.detach().cpu().numpy().astype(np.float64)  # noqa: E731
    h_ref, _, _ = LO.layer_forward(f64(xs[:, :n]), params_np(cell), lap, K, H)
    assert O.normwise_err(f64(hs[:, :n]), h_ref) < TOL


@pytest.mark.parametrize("gates", ["reference", "standard"])
def test_fused_hstep_equals_unfused(dev, gates):
    """The one-launch layer forward + one-launch BPTT steps (hconv='seq':
    cg_lstm_seq_forward / cg_lstm_bwd_step) and the one-launch h-step
    (cg_lstm_hconv_step) against the chebyshev5 + pointwise pair on config E's
    graph at N = 16 (the 2-workgroups-per-sample XCD pairing): states, every
    gradient; both gate sets (each its own sequence-kernel instantiation)."""
    from cnn_graph_amd.gconv_lstm import layer
    Lt, _, M = graph_E()
    T, N, Fin, H, K = 5, 16, 2, 32, 3
    res = {}
    for mode in ("seq", "fused", "unfused"):
        cell, _ = make_cell(Lt, Fin, H, K, gates, dev, seed=41, hconv=mode)
        g = torch.Generator(device=dev)
        g.manual_seed(3)
        xs = torch.randn((T, N, M, Fin), device=dev, generator=g).requires_grad_()
        gh = torch.randn((T, N, M, H), device=dev, generator=g)
        c0 = (torch.randn((N, M, H), device=dev, generator=g) * 0.5).requires_grad_()
        h0 = (torch.randn((N, M, H), device=dev, generator=g) * 0.5).requires_grad_()
        hs, (cT, _) = layer(cell, xs, (c0, h0))
        ((hs * gh).sum() + cT.sum()).backward()
        torch.cuda.synchronize()
        res[mode] = [hs.detach(), cT.detach(), xs.grad, c0.grad, h0.grad] + \
            [p.grad for p in cell.parameters()]
    for mode in ("seq", "fused"):
        for a, b in zip(res[mode], res["unfused"]):
            assert O.normwise_err(a.cpu().numpy(), b.cpu().numpy().astype(np.float64)) < 1e-5, mode
    # the h-conv basis is bit-exact in every mode, so the forward states agree
    # to the contractions' rounding only ('seq' also contracts the x-conv
    # in-kernel, in a different summation order than chebyshev5's GEMM)
    assert O.normwise_err(res["seq"][0].cpu().numpy(), res["fused"][0].cpu().numpy().astype(np.float64)) < 5e-6


@pytest.mark.parametrize("K", [1, 2, 3, 4])
@pytest.mark.parametrize("gates", ["reference", "standard"])
def test_bwd_step_equals_pointwise_plus_cheb_backward(dev, K, gates):
    """cg_lstm_bwd_step (gates backward + dBasis on MFMA + reverse recurrence
    over L~^T in one launch) against lstm_cell_backward + a dx-only
    chebyshev5 backward: dpre and dc_prev bitwise (the same expressions),
    dh_prev within 1e-6; every optional input present and absent.  N = 24:
    XCD pairing on (N % 8 == 0); N = 5: off."""
    from cnn_graph_amd import ops
    from cnn_graph_amd.plan import ChebPlan
    Lt, _, M = graph_E()
    plan = ChebPlan(Lt, device=0)
    H = 32
    for N in (24, 5):
        g = torch.Generator(device=dev)
        g.manual_seed(100 * K + N)
        rn = lambda *sh: torch.randn(sh, device=dev, generator=g)  # noqa: E731
        act = torch.cat([torch.tanh(rn(N, M, H)), torch.sigmoid(rn(N, M, 2 * H)),
                         torch.tanh(rn(N, M, H))], -1).contiguous()
        c_prev, c_out, dh, dh_rec, dc = (rn(N, M, H) for _ in range(5))
        Wh = rn(K * H, 4 * H) * 0.1
        for opt in ((dh, dh_rec, dc, c_prev), (dh, None, None, None), (None, dh_rec, dc, c_prev)):
            a_dh, a_dhr, a_dc, a_cp = opt
            dpre, dcp, dhp = ops.lstm_bwd_step(plan, a_dh, a_dhr, a_dc, act, a_cp, c_out, Wh, K, gates)
            rdpre, rdcp = ops.lstm_cell_backward(a_dh, a_dhr, a_dc, act, a_cp, c_out, H, gates)
            rdhp, _ = ops.cheb_backward(plan, rdpre.view(N, M, 4 * H), None, Wh, K, need_dW=False)
            torch.cuda.synchronize()
            assert torch.equal(dpre, rdpre)
            assert torch.equal(dcp, rdcp)
            assert O.normwise_err(dhp.cpu().numpy(), rdhp.cpu().numpy().astype(np.float64)) < 1e-6
            # the unit-major act records of the sequence kernel: the same step
            act_um = act.view(N, M, 4, H).transpose(-1, -2).contiguous()
            d2, c2, h2 = ops.lstm_bwd_step(plan, a_dh, a_dhr, a_dc, act_um, a_cp, c_out, Wh, K, gates,
                                           act_unit_major=True)
            assert torch.equal(d2, dpre) and torch.equal(c2, dcp) and torch.equal(h2, dhp)
            # no h-conv at the step (dh_prev NULL): the pointwise part alone, on
            # either act layout, bitwise the same dpre / dc_prev
            for a, um in ((act, False), (act_um, True)):
                d3, c3, h3 = ops.lstm_bwd_step(plan, a_dh, a_dhr, a_dc, a, a_cp, c_out, Wh, K, gates,
                                               act_unit_major=um, need_dh_prev=False)
                assert h3 is None and torch.equal(d3, dpre) and torch.equal(c3, dcp)


@pytest.mark.parametrize("gname", ["E", "B", "A"])
@pytest.mark.parametrize("Fin,K", [(2, 3), (1, 2), (5, 3)])
def test_seq_x_basis_prepass_modes_bitwise(dev, cg_opts, Fin, K, gname):
    """The x basis of the one-launch layer forward three ways -- the one-launch
    LDS pre-pass (k_xbasis, CG_OPT_SEQ_XPRE = 1), one streaming launch per order
    (= 2), the recurrence inside k_lstm_seq (= 0).  1 and 2: x planes, hs, cs,
    act and the h planes bitwise equal.  0: the x planes bitwise (the same
    recurrence), the states to fp32 rounding (the in-loop build contracts x in
    another MFMA order than the late x contraction of the pre-pass builds).
    Graphs: E (M = 1024: every lane of the pre-pass's 1024-thread workgroup
    owns a row), B (M = 976, not a multiple of 64) and A (M = 100): lanes past
    the last row must not touch the LDS copy of the basis."""
    from cnn_graph_amd import ops
    from cnn_graph_amd.plan import ChebPlan
    Lt, _, M = graph_E(gname)
    plan = ChebPlan(Lt, device=0)
    T, N, H = 3, 16, 32
    g = torch.Generator(device=dev)
    g.manual_seed(11 * Fin + K)
    xs = torch.rand((T, N, M, Fin), device=dev, generator=g)
    Wx = torch.randn((K * Fin, 4 * H), device=dev, generator=g) * 0.1
    Wh = torch.randn((K * H, 4 * H), device=dev, generator=g) * 0.1
    b = torch.randn((4 * H,), device=dev, generator=g) * 0.1
    R = T * N * M
    out = {}
    for mode in ("1", "2", "0"):
        cg_opts("seq_xpre", mode)
        xpl = torch.full((K, R, Fin), float("nan"), device=dev)
        pl = torch.zeros((max(K - 1, 1), R, H), device=dev)  # (step 0 has no h-conv: untouched)
        act_t = torch.empty((R, 4 * H), device=dev)
        hs, cs, act, _ = ops.lstm_seq_forward_x(plan, xs, Wx, Wh, b, K, out_act=act_t, planes=pl[0],
                                                plane_stride=R * H, xplanes=xpl)
        torch.cuda.synchronize()
        out[mode] = (xpl, hs, cs, act, pl)
    for a, c in zip(out["1"], out["2"]):
        assert torch.equal(a, c)
    assert torch.equal(out["1"][0], out["0"][0])
    for a, c in zip(out["1"][1:], out["0"][1:]):
        # fp32 rounding of another MFMA order (1.0e-6 measured on graph B)
        err = O.normwise_err(a.cpu().numpy(), c.cpu().numpy().astype(np.float64))
        assert err < 4e-6, err
    assert ops.lstm_seq_fault(plan, wait=True) is False


def test_seq_forward_more_samples_than_pairs(dev):
    """N = 136 > the 128 workgroup pairs of a 256-CU chip: pairs take a second
    sample in turn (XCD pairing on).  States and planes equal the per-step
    one-launch h-step path; no hand-off timed out."""
    from cnn_graph_amd import ops
    from cnn_graph_amd.gconv_lstm import layer
    Lt, _, M = graph_E()
    T, N, Fin, H, K = 3, 136, 2, 32, 3
    res = {}
    for mode in ("seq", "fused"):
        cell, _ = make_cell(Lt, Fin, H, K, "reference", dev, seed=43, hconv=mode)
        g = torch.Generator(device=dev)
        g.manual_seed(5)
        xs = torch.randn((T, N, M, Fin), device=dev, generator=g)
        c0 = torch.randn((N, M, H), device=dev, generator=g) * 0.5
        h0 = torch.randn((N, M, H), device=dev, generator=g) * 0.5
        with torch.no_grad():
            hs, (cT, _) = layer(cell, xs, (c0, h0))
        res[mode] = (hs, cT)
        if mode == "seq":  # explicit calls with the status check
            assert cell.seq_x  # the layer fuses the x-conv in: same launch as _x
            hs1 = ops.lstm_seq_forward_x(cell.plan, xs, cell.Wx.detach(), cell.Wh.detach(),
                                         cell.b.detach(), K, "reference", h0=h0, c0=c0,
                                         check=True)[0]
            assert torch.equal(hs1.view_as(hs), hs)
            _, gx = ops.cheb_forward(cell.plan, xs.view(T * N, M, Fin), cell.Wx.detach(), K)
            hs2, cs2, _ = ops.lstm_seq_forward(cell.plan, gx, cell.Wh.detach(), cell.b.detach(), K,
                                               T, N, "reference", h0=h0, c0=c0, check=True)
            assert O.normwise_err(hs2.cpu().numpy(), hs.cpu().numpy().astype(np.float64)) < TOL
    torch.cuda.synchronize()
    for a, b in zip(res["seq"], res["fused"]):  # contraction summed in another order
        assert O.normwise_err(a.cpu().numpy(), b.cpu().numpy().astype(np.float64)) < TOL


def test_config_E_full_batch_gradients_vs_oracle(dev):
    """Config E at full size (M = 1024, T = 12, K = 3, Fin = 2, H = 32,
    N = 128 per GPU) through the one-launch layer forward and BPTT steps, with
    a loss that reads 3 samples only (the filter is per-sample independent):
    every gradient -- dWx, dWh, db over the whole batch, dx of those samples --
    against the float64 oracle run on the 3 samples (not against cell
    stepping); dx of every other sample exactly 0."""
    from cnn_graph_amd.gconv_lstm import layer
    Lt, _, M = graph_E()
    T, N, Fin, H, K = 12, 128, 2, 32, 3
    cell, L = make_cell(Lt, Fin, H, K, "reference", dev, seed=51)
    assert cell.seq
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    xs = torch.rand((T, N, M, Fin), device=dev, generator=g)
    sel = [3, 64, 127]
    gh = torch.zeros((T, N, M, H), device=dev)
    gsel = torch.randn((T, len(sel), M, H), device=dev, generator=g)
    gh[:, sel] = gsel
    xa = xs.clone().requires_grad_()
    hs, _ = layer(cell, xa)
    (hs * gh).sum().backward()
    torch.cuda.synchronize()
    f64 = lambda a: a.detach().cpu().numpy().astype(np.float64)  # noqa: E731
    lap = oracle_lap(cell, L)
    p = params_np(cell)
    h_ref, _, caches = LO.layer_forward(f64(xs[:, sel]), p, lap, K, H)
    assert O.normwise_err(f64(hs[:, sel]), h_ref) < TOL
    dxs, _, _, dWx, dWh, db = LO.layer_backward(f64(gsel), None, caches, p, lap, K, H)
    for name, got, ref in (("dWx", cell.Wx.grad, dWx), ("dWh", cell.Wh.grad, dWh),
                           ("db", cell.b.grad, db), ("dx", xa.grad[:, sel], dxs)):
        err = O.normwise_err(f64(got), ref)
        assert err < TOL, (name, err)
    rest = [i for i in range(N) if i not in sel]
    assert int(torch.count_nonzero(xa.grad[:, rest])) == 0


@pytest.mark.timeout(600)
def test_config_E_every_sample_vs_oracle(dev):
    """Config E at full size with a loss over all N = 128 samples: hs of every
    sample and every gradient (dWx, dWh, db over the batch, dx of every
    sample) against the float64 oracle run on the whole batch (~30 s of
    numpy), through the one-launch layer forward and BPTT steps."""
    from cnn_graph_amd.gconv_lstm import layer
    Lt, _, M = graph_E()
    T, N, Fin, H, K = 12, 128, 2, 32, 3
    cell, L = make_cell(Lt, Fin, H, K, "reference", dev, seed=53)
    assert cell.seq
    g = torch.Generator(device=dev)
    g.manual_seed(9)
    xs = torch.rand((T, N, M, Fin), device=dev, generator=g)
    gh = torch.randn((T, N, M, H), device=dev, generator=g)
    xa = xs.clone().requires_grad_()
    hs, _ = layer(cell, xa)
    (hs * gh).sum().backward()
    torch.cuda.synchronize()
    f64 = lambda a: a.detach().cpu().numpy().astype(np.float64)  # noqa: E731
    lap = oracle_lap(cell, L)
    p = params_np(cell)
    h_ref, _, caches = LO.layer_forward(f64(xs), p, lap, K, H)
    assert O.normwise_err(f64(hs), h_ref) < TOL
    dxs, _, _, dWx, dWh, db = LO.layer_backward(f64(gh), None, caches, p, lap, K, H)
    for name, got, ref in (("dWx", cell.Wx.grad, dWx), ("dWh", cell.Wh.grad, dWh),
                           ("db", cell.b.grad, db), ("dx", xa.grad, dxs)):
        err = O.normwise_err(f64(got), ref)
        assert err < TOL, (name, err)


@pytest.mark.parametrize("Fin,K", [(2, 3), (1, 1), (8, 4), (5, 2)])
def test_lstm_weight_grads_one_pass(dev, Fin, K):
    """cg_lstm_weight_grads (dWh, dWx and db of a layer in one pass over dpre)
    against the per-weight kernels: dWh and dWx bitwise equal to
    cg_weight_grad_planes (same chunks, same per-tile row order), db within
    1e-6 of cg_bias_grad (ones column on the MFMA vs a column-sum kernel), and
    all three against float64."""
    from cnn_graph_amd import ops
    H, R = 32, 3 * 1021
    g = torch.Generator(device=dev)
    g.manual_seed(7 * Fin + K)
    hst, xst = R * H + 96, R * Fin + 40
    hbuf = torch.randn((K * hst,), device=dev, generator=g)
    xbuf = torch.randn((K * xst,), device=dev, generator=g)
    dpre = torch.randn((R, 4 * H), device=dev, generator=g)
    hpl, xpl = hbuf[:R * H].view(R, H), xbuf[:R * Fin].view(R, Fin)
    dWh, dWx, db = ops.lstm_weight_grads(hpl, hst, xpl, xst, K, R, dpre)
    rWh = ops.weight_grad_planes(hpl, hst, K, R, dpre)
    rWx = ops.weight_grad_planes(xpl, xst, K, R, dpre)
    rdb = ops.bias_grad(dpre)
    torch.cuda.synchronize()
    assert torch.equal(dWh, rWh)
    assert torch.equal(dWx, rWx)
    assert O.normwise_err(db.cpu().numpy(), rdb.cpu().numpy().astype(np.float64)) < 1e-6
    d64 = dpre.double().cpu()
    for buf, st, w, got in ((hbuf, hst, H, dWh), (xbuf, xst, Fin, dWx)):
        pl = torch.stack([buf[k * st:k * st + R * w].view(R, w) for k in range(K)]).double().cpu()
        ref = torch.einsum("krc,rg->ckg", pl, d64).reshape(w * K, 4 * H)
        assert O.normwise_err(got.cpu().numpy(), ref.numpy()) < 1e-5
    assert O.normwise_err(db.cpu().numpy(), d64.sum(0).numpy()) < 1e-5


def test_seq_handoff_timeout_raises_and_poisons(dev):
    """A lost pair hand-off (fault injected: workgroup 0 of pair 0 stops
    publishing its step counter from step 1, cg_plan_set_seq_fault_test) ends the
    launch after the 2 s timeout instead of hanging, and no caller can consume
    its outputs: every hs / cs entry the lost workgroups owed is NaN, an
    inference layer() raises CGError, a training layer()'s backward raises
    before forming any gradient, and the plan works again afterwards."""
    from cnn_graph_amd import _lib, ops
    from cnn_graph_amd.gconv_lstm import layer
    Lt, _, M = graph_E()
    T, N, Fin, H, K = 3, 4, 2, 32, 3
    cell, _ = make_cell(Lt, Fin, H, K, "reference", dev, seed=61)
    assert cell.seq
    g = torch.Generator(device=dev)
    g.manual_seed(9)
    xs = torch.rand((T, N, M, Fin), device=dev, generator=g)
    with torch.no_grad():
        ref, _ = layer(cell, xs)
    torch.cuda.synchronize()
    assert bool(torch.isfinite(ref).all())
    cell.plan.set_seq_fault_test(1)
    with torch.no_grad():
        with pytest.raises(_lib.CGError, match="hand-off timed out"):
            layer(cell, xs)
    # the explicit call: the poisoned entries.  Pair 0 (sample 0): workgroup 1
    # (units 16..31) times out at step 1, workgroup 0 (units 0..15) at step 2
    hs, cs, _, _ = ops.lstm_seq_forward_x(cell.plan, xs, cell.Wx.detach(), cell.Wh.detach(),
                                          cell.b.detach(), K, "reference")
    with pytest.raises(_lib.CGError):
        ops.lstm_seq_fault(cell.plan, wait=True)
    for a in (hs, cs):
        assert bool(torch.isnan(a[1, 0, :, 16:]).all()) and bool(torch.isnan(a[2, 0]).all())
        assert bool(torch.isfinite(a[0]).all()) and bool(torch.isfinite(a[:, 1:]).all())
        assert bool(torch.isfinite(a[1, 0, :, :16]).all())
    assert torch.equal(hs[:, 1:], ref[:, 1:])
    # training: the forward returns, its backward refuses
    hs2, _ = layer(cell, xs)
    with pytest.raises(_lib.CGError, match="hand-off timed out"):
        hs2.sum().backward()
    cell.plan.set_seq_fault_test(-1)
    assert ops.lstm_seq_fault(cell.plan, wait=True) is False  # reported once, then reset
    with torch.no_grad():
        again, _ = layer(cell, xs)
    assert torch.equal(again, ref)
