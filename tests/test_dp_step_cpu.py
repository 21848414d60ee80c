"""The data-parallel step schedule bench.py times (cnn_graph_amd/dp_step.py),
checked on the CPU with a recording stand-in for the C-ABI runner: which
weights each forward and backward sees, where the exchange and the Adam
updates sit, and that every schedule applies updates 1..n in order
(lib/graph_model.py:277-298: compute_gradients -> exchange -> apply_gradients).
The numerics of the same schedule on the GPU at world size 2:
tests/test_gpu_dp_bench.py."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
torch = pytest.importorskip("torch")


class Rec:
    """Runner stand-in: records the calls; weights are identified by object."""

    def __init__(self):
        self.log = []
        self.dW = torch.zeros(3)

    def forward(self, x, W, stream=None):
        self.log.append(("fwd", id(W)))

    def forward_adam(self, x, W, grad, m, v, W_out, m_out, v_out, step, lr, b1, b2, eps,
                     grad_scale=1.0, stream=None):
        assert grad is self.dW
        self.log.append(("fwd_adam", id(W), id(W_out), step, grad_scale))

    def backward(self, dy, W, need_dx=True, stream=None):
        self.log.append(("bwd", id(W)))

    def backward_adam(self, dy, W, m, v, step, lr, b1, b2, eps, grad_scale=1.0, need_dx=True,
                      stream=None):
        self.log.append(("bwd_adam", id(W), step, grad_scale))


def make(schedule, world=1, allreduce=True, monkeypatch=None):
    from cnn_graph_amd import dp_step
    monkeypatch.setattr(dp_step._lib, "lib", lambda: type("L", (), {"cg_adam_update": None})())
    r = Rec()
    ar = (lambda s: r.log.append(("allreduce",))) if allreduce else None
    tr = dp_step.ChebTrainStep(r, None, None, torch.zeros(3), world=world, allreduce=ar,
                               schedule=schedule)
    monkeypatch.setattr(tr, "_adam_update",
                        lambda W, m, v, step, s: r.log.append(("adam", id(W), step)))
    return r, tr


def test_forward_applied_adam_schedule(monkeypatch):
    r, tr = make("auto", world=4, monkeypatch=monkeypatch)
    assert tr.schedule == "forward" and tr.scale == 0.25
    W0, W1 = (id(w) for w in tr.W)
    for i in range(3):
        tr.step(i, 0)
    Wfin = tr.finish(3, 0)
    assert r.log == [
        ("fwd", W0), ("bwd", W0), ("allreduce",),
        ("fwd_adam", W0, W1, 1, 0.25), ("bwd", W1), ("allreduce",),   # update 1 by step 1's forward
        ("fwd_adam", W1, W0, 2, 0.25), ("bwd", W0), ("allreduce",),   # update 2
        ("adam", W0, 3)]                                               # update 3 by finish
    assert id(Wfin) == W0


def test_fused_and_unfused_schedules(monkeypatch):
    r, tr = make("auto", world=1, allreduce=False, monkeypatch=monkeypatch)
    assert tr.schedule == "fused" and tr.scale == 1.0
    W0 = id(tr.W[0])
    for i in range(2):
        tr.step(i, 0)
    assert tr.finish(2, 0) is tr.W[0]
    assert r.log == [("fwd", W0), ("bwd_adam", W0, 1, 1.0), ("fwd", W0), ("bwd_adam", W0, 2, 1.0)]
    r, tr = make("unfused", world=2, monkeypatch=monkeypatch)
    W0 = id(tr.W[0])
    for i in range(2):
        tr.step(i, 0)
    assert r.log == [("fwd", W0), ("bwd", W0), ("allreduce",), ("adam", W0, 1),
                     ("fwd", W0), ("bwd", W0), ("allreduce",), ("adam", W0, 2)]


def test_schedule_argument_errors(monkeypatch):
    with pytest.raises(ValueError):
        make("fused", world=2, allreduce=True, monkeypatch=monkeypatch)
    with pytest.raises(ValueError):
        make("bogus", monkeypatch=monkeypatch)
