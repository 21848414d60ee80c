"""gconvRNN.Model._build_optim's update rules (lib/gconvRNN.py:381-389) on the
HIP kernels against float64 restatements of TF 1.x's training ops:
GradientDescent (ApplyGradientDescent) and RMSProp (ApplyRMSProp, not
centered; ms starts at ones), with the grad_scale of the data-parallel
exchange, over several steps (RMSProp with and without momentum)."""
import numpy as np
import pytest

from oracle import cheb_oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev(built_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


def _grads(n, steps, seed):
    rng = np.random.default_rng(seed)
    return [rng.standard_normal(n).astype(np.float32) for _ in range(steps)]


@pytest.mark.parametrize("n", [1, 1000, 70001])
def test_sgd_update_vs_float64(dev, n):
    from cnn_graph_amd import ops
    rng = np.random.default_rng(n)
    p0 = rng.standard_normal(n).astype(np.float32)
    p = torch.from_numpy(p0).to(dev)
    ref = p0.astype(np.float64)
    for g in _grads(n, 4, n + 1):
        ops.sgd_update(p, torch.from_numpy(g).to(dev), lr=0.05, grad_scale=0.25)
        ref = ref - (g.astype(np.float64) * 0.25) * 0.05
    assert O.normwise_err(p.cpu().numpy(), ref) < 1e-6


@pytest.mark.parametrize("momentum", [0.0, 0.9])
def test_rmsprop_update_vs_float64(dev, momentum):
    from cnn_graph_amd import ops
    n = 40000
    rng = np.random.default_rng(7)
    p0 = rng.standard_normal(n).astype(np.float32)
    p = torch.from_numpy(p0).to(dev)
    ms = torch.ones(n, device=dev)
    mom = torch.zeros(n, device=dev)
    ref, rms, rmom = p0.astype(np.float64), np.ones(n), np.zeros(n)
    for g in _grads(n, 5, 8):
        ops.rmsprop_update(p, torch.from_numpy(g).to(dev), ms, mom, lr=1e-2, rho=0.9,
                           momentum=momentum, eps=1e-10, grad_scale=0.5)
        g64 = g.astype(np.float64) * 0.5
        rms = rms + (g64 * g64 - rms) * 0.1
        rmom = rmom * momentum + g64 * 1e-2 / np.sqrt(rms + 1e-10)
        ref = ref - rmom
    torch.cuda.synchronize()
    assert O.normwise_err(ms.cpu().numpy(), rms) < 1e-6
    assert O.normwise_err(mom.cpu().numpy(), rmom) < 1e-6
    assert O.normwise_err(p.cpu().numpy(), ref) < 1e-6
