"""Config E's 4-GPU split (BASELINE configs[4]: gconv-LSTM, batch 512 over
4 x MI355X) as a data-parallel training step: gconv_lstm.GLSTMModel
(inference_glstm = glstm_layer + fc_layer, lib/gconv_lstm.py:271-281, :609-636;
MSE + Adam, lib/graph_model.py:246-310) with ONE all-reduce of the flat
gradient bucket (every layer's Wx, Wh, b and the fc weight, 53.5 KB) per step
and grad_scale = 1/world (lib/graph_model.py:296-298 is where the exchange sits).

Two ranks share this box's GPU over gloo (RCCL refuses two ranks on one device)
at config E's graph and shape (T = 12, K = 3, H = 32, Fin = 2) with 4 samples
per rank; one process trains on the whole 8-sample batch.  Bars: both replicas
bitwise equal after every step; the first step's exchanged gradient (sum / 2)
within 1e-5 (normwise) of the full batch's, and the parameters within 1e-5 of
the full-batch run's after each of 3 Adam steps."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT
from oracle import cheb_oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev(built_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)


@pytest.mark.timeout(400)
def test_glstm_dp_world2_matches_full_batch(dev, tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import glstm_dp_worker as Wk
    out = tmp_path / "glstm_dp.npz"
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "tests", "glstm_dp_worker.py"), str(out)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=360)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    d = np.load(out)
    assert int(d["world"]) == 2
    assert np.array_equal(d["P"], d["P_r1"]), "replicas diverged"
    L, x, labels = Wk.problem()
    P, g1, losses = Wk.run(L, x, labels, dev, None)
    assert np.all(np.isfinite(losses))
    assert O.normwise_err(d["g1"], g1.astype(np.float64)) < 1e-5
    for n in range(Wk.STEPS):
        if n:
            assert not np.array_equal(d["P"][n], d["P"][n - 1])  # the update ran
        err = O.normwise_err(d["P"][n], P[n].astype(np.float64))
        assert err < 1e-5, (n + 1, err)


def test_glstm_model_flat_bucket_and_optimizers(dev):
    """The flat buffers: every parameter aliases the flat buffer and its .grad
    the flat bucket after a step (autograd accumulated in place); 53.5 KB at
    config E; the fc output shape; sgd / rmsprop run and move the weights by
    their own rules (one step from the same start: sgd moves by lr * g,
    rmsprop by lr * g / sqrt(0.1 g^2 + 0.9 + 1e-10))."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import glstm_dp_worker as Wk
    from cnn_graph_amd.gconv_lstm import GLSTMModel
    L, x, labels = Wk.problem()
    x, labels = x[:2], labels[:2]
    xs, ys = torch.from_numpy(x).to(dev), torch.from_numpy(labels).to(dev)
    res = {}
    for opt in ("adam", "sgd", "rmsprop"):
        m = GLSTMModel(L, 2, Wk.T, Wk.FIN, num_hidden=Wk.H, K=Wk.K, out_features=Wk.FOUT, keep_prob=1.0,
                       optimizer=opt, learning_rate=1e-2, device=dev, seed=5)
        assert m.flat.numel() * 4 == 53504
        p0 = m.flat.clone()
        out = m.forward(xs)
        assert tuple(out.shape) == (2, m.M, Wk.FOUT)
        m.train_step(xs, ys)
        torch.cuda.synchronize()
        for p in m.params:
            assert p.data_ptr() >= m.flat.data_ptr()
            assert m.grad.data_ptr() <= p.grad.data_ptr() < m.grad.data_ptr() + 4 * m.grad.numel()
        res[opt] = (p0.double().cpu(), m.flat.double().cpu(), m.grad.double().cpu())
    for opt in ("adam", "sgd", "rmsprop"):
        assert torch.equal(res[opt][0], res["adam"][0])  # same seed, same start
        assert torch.equal(res[opt][2], res["adam"][2])  # same first gradient
    p0, _, g = res["sgd"]
    assert O.normwise_err(res["sgd"][1].numpy(), (p0 - 1e-2 * g).numpy()) < 1e-6
    ms = 1.0 + (g * g - 1.0) * 0.1
    ref = p0 - 1e-2 * g / torch.sqrt(ms + 1e-10)
    assert O.normwise_err(res["rmsprop"][1].numpy(), ref.numpy()) < 1e-6


def test_glstm_dropout_reproducible_from_seed(dev):
    """keep_prob < 1 (the reference default 0.8, lib/gconv_lstm.py:616): the
    dropout masks derive from (model seed, rank, layer), so two
    models built with one seed train bitwise identically whatever was built
    before them in the process, another seed (or another rank) draws other
    masks, and the masks really drop (the step differs from keep_prob = 1)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import glstm_dp_worker as Wk
    from cnn_graph_amd.gconv_lstm import GLSTMModel, dropout_seed
    L, x, labels = Wk.problem()
    xs, ys = torch.from_numpy(x[:2]).to(dev), torch.from_numpy(labels[:2]).to(dev)

    class Rank:  # a comm stand-in that names a rank (world 1: no exchange)
        def __init__(self, r):
            self.rank, self.world = r, 1

    def train(seed, keep, comm=None):
        m = GLSTMModel(L, 2, Wk.T, Wk.FIN, num_hidden=Wk.H, K=Wk.K, out_features=Wk.FOUT,
                       layer_count=2, keep_prob=keep, device=dev, seed=seed, comm=comm)
        for _ in range(2):
            m.train_step(xs, ys)
        torch.cuda.synchronize()
        return m.flat.cpu().clone()

    a = train(7, 0.8)
    train(9, 0.8)  # more wrappers created in between: must not shift the next model's masks
    b = train(7, 0.8)
    assert torch.equal(a, b)
    assert not torch.equal(a, train(8, 0.8))
    assert not torch.equal(a, train(7, 0.8, Rank(1)))
    assert not torch.equal(a, train(7, 1.0))
    assert torch.equal(a, train(7, 0.8, Rank(0)))
    seeds = {dropout_seed(7, r, li) for r in range(8) for li in range(4)}
    assert len(seeds) == 32 and all(0 <= s < 2 ** 64 for s in seeds)
