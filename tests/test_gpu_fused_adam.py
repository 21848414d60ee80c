"""cg_cheb_backward_adam: the one-GPU training step's Adam update applied by the
dW slab reduction (lib/graph_model.py:277-298, compute_gradients +
apply_gradients with no exchange in between).  Bar: dW and dx BITWISE equal to
cg_cheb_backward + cg_adam_update every step (both Adam kernels share one
element function compiled with fp contraction off, so W, m, v are bitwise
equal too), with and without dx, and the fused W within 1e-5 of the float64
Adam restatement."""
import ctypes

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


def adam64(W, g, m, v, step, lr=1e-3, b1=0.9, b2=0.999, eps=1e-8):
    """TF-1.x AdamOptimizer update (float64), the rule k_adam implements."""
    lr_t = lr * np.sqrt(1 - b2 ** step) / (1 - b1 ** step)
    m = m + (g - m) * (1 - b1)
    v = v + (g * g - v) * (1 - b2)
    return W - lr_t * m / (np.sqrt(v) + eps), m, v


@pytest.mark.parametrize("need_dx", [True, False])
@pytest.mark.parametrize("name,path", [("golden_A.npz", "resident"), ("golden_B.npz", "resident"),
                                       ("golden_E.npz", "stream")])
def test_backward_adam_matches_unfused(dev, name, path, need_dx):
    from cnn_graph_amd import _lib, ops
    from cnn_graph_amd.plan import ChebPlan
    c = case(load_golden(name))
    M, N, Fin, K, Fout = c["M"], c["N"], c["Fin"], c["K"], c["Fout"]
    Lt = scipy.sparse.csr_matrix((c["Lt_val"], c["Lt_col"], c["Lt_rowptr"]), shape=(M, M))
    plan = ChebPlan(Lt, device=0, path=path)
    x = torch.from_numpy(np.ascontiguousarray(c["x"], dtype=np.float32)).to(dev)
    dy = torch.from_numpy(np.ascontiguousarray(c["dy"], dtype=np.float32)).to(dev)
    W0 = torch.from_numpy(np.ascontiguousarray(c["W"], dtype=np.float32)).to(dev)
    ra, rb = ops.ChebRunner(plan, N, Fin, K, Fout, dev), ops.ChebRunner(plan, N, Fin, K, Fout, dev)
    Wa, Wb = W0.clone(), W0.clone()
    ma, va, mb, vb = (torch.zeros_like(W0) for _ in range(4))
    adam = _lib.lib().cg_adam_update
    W64, m64, v64 = (f.astype(np.float64) for f in (c["W"], np.zeros_like(c["W"]), np.zeros_like(c["W"])))
    for step in (1, 2, 3):
        ra.forward(x, Wa)
        rb.forward(x, Wb)
        dxa, dWa = ra.backward_adam(dy, Wa, ma, va, step, need_dx=need_dx)
        dxb, dWb = rb.backward(dy, Wb, need_dx=need_dx)
        torch.cuda.synchronize()
        assert torch.equal(dWa, dWb), "fused reduction changed dW"
        if need_dx:
            assert torch.equal(dxa, dxb)
        else:
            assert dxa is None and dxb is None
        g64 = dWb.cpu().numpy().astype(np.float64)
        _lib.check("cg_adam_update", adam(Wb.data_ptr(), dWb.data_ptr(), mb.data_ptr(), vb.data_ptr(),
                                          Wb.numel(), ctypes.c_float(1e-3), ctypes.c_float(0.9),
                                          ctypes.c_float(0.999), ctypes.c_float(1e-8), step,
                                          ctypes.c_float(1.0), None))
        W64, m64, v64 = adam64(W64, g64, m64, v64, step)
        torch.cuda.synchronize()
        for a, b in ((Wa, Wb), (ma, mb), (va, vb)):
            assert torch.equal(a, b), "fused Adam differs from cg_adam_update"
        assert O.normwise_err(Wa.cpu().numpy(), W64) < 1e-5



@pytest.mark.parametrize("name,path", [("golden_B.npz", "resident"), ("golden_E.npz", "resident"),
                                       ("golden_E.npz", "stream")])
def test_forward_adam_matches_adam_then_forward(dev, name, path):
    """cg_cheb_forward_adam (the exchange step's Adam applied by the next
    forward, out of place): W', m', v' and y bitwise equal to cg_adam_update on
    copies followed by the plain forward, over three steps (fast kernels'
    prologue and, on the streaming path, the k_adam + forward sequence)."""
    from cnn_graph_amd import _lib, ops
    from cnn_graph_amd.plan import ChebPlan
    c = case(load_golden(name))
    M, N, Fin, K, Fout = c["M"], c["N"], c["Fin"], c["K"], c["Fout"]
    Lt = scipy.sparse.csr_matrix((c["Lt_val"], c["Lt_col"], c["Lt_rowptr"]), shape=(M, M))
    plan = ChebPlan(Lt, device=0, path=path)
    x = torch.from_numpy(np.ascontiguousarray(c["x"], dtype=np.float32)).to(dev)
    dy = torch.from_numpy(np.ascontiguousarray(c["dy"], dtype=np.float32)).to(dev)
    W0 = torch.from_numpy(np.ascontiguousarray(c["W"], dtype=np.float32)).to(dev)
    ra, rb = ops.ChebRunner(plan, N, Fin, K, Fout, dev), ops.ChebRunner(plan, N, Fin, K, Fout, dev)
    Wa, ma, va = W0.clone(), torch.zeros_like(W0), torch.zeros_like(W0)
    Wb = [W0.clone(), torch.empty_like(W0)]
    mb = [torch.zeros_like(W0), torch.empty_like(W0)]
    vb = [torch.zeros_like(W0), torch.empty_like(W0)]
    adam = _lib.lib().cg_adam_update
    scale = 0.5
    ra.forward(x, Wa)
    rb.forward(x, Wb[0])
    for step in (1, 2, 3):
        ra.backward(dy, Wa)
        rb.backward(dy, Wb[(step - 1) % 2])
        torch.cuda.synchronize()
        assert torch.equal(ra.dW, rb.dW)
        _lib.check("cg_adam_update", adam(Wa.data_ptr(), ra.dW.data_ptr(), ma.data_ptr(),
                                          va.data_ptr(), Wa.numel(), ctypes.c_float(1e-3),
                                          ctypes.c_float(0.9), ctypes.c_float(0.999),
                                          ctypes.c_float(1e-8), step, ctypes.c_float(scale), None))
        ra.forward(x, Wa)
        p, q = (step - 1) % 2, step % 2
        rb.forward_adam(x, Wb[p], rb.dW, mb[p], vb[p], Wb[q], mb[q], vb[q], step, grad_scale=scale)
        torch.cuda.synchronize()
        for a_, b_ in ((Wa, Wb[q]), (ma, mb[q]), (va, vb[q]), (ra.y, rb.y)):
            assert torch.equal(a_, b_), "forward_adam differs from adam + forward"
    # the outputs may not alias the inputs
    with pytest.raises(_lib.CGError):
        rb.forward_adam(x, Wb[0], rb.dW, mb[0], vb[0], Wb[0], mb[1], vb[1], 4)
