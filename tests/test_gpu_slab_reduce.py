"""The dW slab reduction after the fused-dW fast backward (k_reduce_slabs /
k_reduce_slabs_adam): dW must be BITWISE the fixed-order sum over the
per-sample slabs the kernel leaves in the workspace (class c = n mod 16
summed in increasing n from +0, then the 16 class sums in order), for full,
ragged and tiny batches, on repeated and interleaved calls, and with the Adam
step riding on it; and within 1e-5 of the float64 dW = basis^T dy
(lib/graph_model.py:296, TF autodiff of lib/graph_conv.py:175).

(An in-kernel variant -- the last workgroups to finish reduce the slabs in
cheb_bwd_fast's tail by arrival counting -- passed these tests and was
measured 6-9 us slower per backward than the separate launch on MI355X:
profiles/r02_tail.)"""
import numpy as np
import pytest
import scipy.sparse

from conftest import case, load_golden

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev(built_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from cnn_graph_amd import _lib
    _lib.lib()
    return torch.device("cuda", 0)


@pytest.fixture(scope="module")
def plan_B(dev):
    from cnn_graph_amd.plan import ChebPlan
    c = case(load_golden("golden_B.npz"))
    M = c["M"]
    Lt = scipy.sparse.csr_matrix((c["Lt_val"], c["Lt_col"], c["Lt_rowptr"]), shape=(M, M))
    return ChebPlan(Lt, device=0, path="resident"), c


def class_order_sum(slabs):
    """k_reduce_slabs' order in float32 (IEEE adds, elementwise)."""
    N = slabs.shape[0]
    parts = []
    for q in range(16):
        s = np.zeros(slabs.shape[1:], np.float32)
        for z in range(q, N, 16):
            s = s + slabs[z]
        parts.append(s)
    t = np.zeros(slabs.shape[1:], np.float32)
    for q in range(16):
        t = t + parts[q]
    return t


@pytest.mark.parametrize("N", [1, 5, 16, 17, 40, 256])
def test_slab_reduction_bitwise(dev, plan_B, N):
    from cnn_graph_amd import ops
    plan, c = plan_B
    M, Fin, K, Fout = c["M"], c["Fin"], c["K"], c["Fout"]
    assert plan.query_path(N, Fin, K, Fout) == "resident"
    g = torch.Generator().manual_seed(1234 + N)
    x = torch.randn((N, M, Fin), generator=g).to(dev)
    W = (0.1 * torch.randn((Fin * K, Fout), generator=g)).to(dev)
    r = ops.ChebRunner(plan, N, Fin, K, Fout, dev)
    r.forward(x, W)
    for rep in range(3):
        dy = torch.randn((N, M, Fout), generator=g).to(dev)
        _, dW = r.backward(dy, W)
        torch.cuda.synchronize()
        slabs = r.ws[: N * Fin * K * Fout * 4].view(torch.float32).view(N, Fin * K, Fout)
        want = class_order_sum(slabs.cpu().numpy())
        assert np.array_equal(dW.cpu().numpy(), want), f"rep {rep}: slab sum order differs"
        b64 = r.basis.cpu().numpy().astype(np.float64)
        d64 = dy.cpu().numpy().astype(np.float64).reshape(N * M, Fout)
        ref = b64.T @ d64
        assert np.abs(dW.cpu().numpy() - ref).max() / np.abs(ref).max() < 1e-5


def test_slab_reduction_interleaved_batches(dev, plan_B):
    """Two runners of different N on one plan, alternating: every call
    reproduces its first result bitwise."""
    from cnn_graph_amd import ops
    plan, c = plan_B
    M, Fin, K, Fout = c["M"], c["Fin"], c["K"], c["Fout"]
    g = torch.Generator().manual_seed(7)
    runs = []
    for N in (33, 256):
        x = torch.randn((N, M, Fin), generator=g).to(dev)
        dy = torch.randn((N, M, Fout), generator=g).to(dev)
        W = (0.1 * torch.randn((Fin * K, Fout), generator=g)).to(dev)
        r = ops.ChebRunner(plan, N, Fin, K, Fout, dev)
        r.forward(x, W)
        runs.append((r, dy, W))
    first = []
    for r, dy, W in runs:
        first.append(r.backward(dy, W)[1].clone())
    for it in range(4):
        for (r, dy, W), d0 in zip(runs, first):
            assert torch.equal(r.backward(dy, W)[1], d0), f"iteration {it}"


def test_reduce_adam_matches_two_launch_adam(dev, plan_B):
    """backward_adam (reduction + Adam in one launch) vs backward +
    cg_adam_update at N = 100: W, m, v, dW bitwise, over 3 steps."""
    import ctypes

    from cnn_graph_amd import _lib, ops
    plan, c = plan_B
    M, Fin, K, Fout = c["M"], c["Fin"], c["K"], c["Fout"]
    N = 100
    g = torch.Generator().manual_seed(11)
    x = torch.randn((N, M, Fin), generator=g).to(dev)
    dy = torch.randn((N, M, Fout), generator=g).to(dev)
    W0 = (0.1 * torch.randn((Fin * K, Fout), generator=g)).to(dev)
    ra, rb = ops.ChebRunner(plan, N, Fin, K, Fout, dev), ops.ChebRunner(plan, N, Fin, K, Fout, dev)
    Wa, Wb = W0.clone(), W0.clone()
    ma, va, mb, vb = (torch.zeros_like(W0) for _ in range(4))
    adam = _lib.lib().cg_adam_update
    for step in (1, 2, 3):
        ra.forward(x, Wa)
        rb.forward(x, Wb)
        _, dWa = ra.backward_adam(dy, Wa, ma, va, step)
        _, dWb = rb.backward(dy, Wb)
        _lib.check("cg_adam_update", adam(Wb.data_ptr(), dWb.data_ptr(), mb.data_ptr(), vb.data_ptr(),
                                          Wb.numel(), ctypes.c_float(1e-3), ctypes.c_float(0.9),
                                          ctypes.c_float(0.999), ctypes.c_float(1e-8), step,
                                          ctypes.c_float(1.0), None))
        torch.cuda.synchronize()
        assert torch.equal(dWa, dWb)
        for a_, b_ in ((Wa, Wb), (ma, mb), (va, vb)):
            assert torch.equal(a_, b_)
