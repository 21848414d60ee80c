"""Data parallelism of the training step with the HIP kernels at world size 2
(the exchange sits between compute_gradients and
apply_gradients, lib/graph_model.py:296-298): two ranks, each running
ResGNN.train_step on its half of a fixed batch with ONE all-reduce of the flat
gradient buffer per step (dist.TorchComm over gloo: both ranks share this
box's one GPU, which RCCL does not allow), against one process training on the
whole batch.  Bars: the exchanged gradient / world and the loss within 1e-5
normwise of the full-batch ones, both replicas bitwise identical after three
steps, and their parameters within 1e-4 of the full-batch run's (Adam's
normalised step amplifies fp32 reduction-order differences)."""
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


@pytest.mark.timeout(300)
def test_resgnn_dp_world2_matches_full_batch(dev, tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import dp_resgnn_worker as Wk
    out = tmp_path / "dp.npz"
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "tests", "dp_resgnn_worker.py"), str(out)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    d = np.load(out)
    L, x, labels = Wk.problem()
    losses, g1, flat = Wk.run(Wk.N_GLOBAL, x, labels, L, None, dev)
    assert np.array_equal(d["flat"], d["flat_r1"]), "replicas diverged"
    assert O.normwise_err(d["loss"], losses) < 1e-5
    assert O.normwise_err(d["grad1"], g1) < 1e-5
    assert O.normwise_err(d["flat"], flat) < 1e-4
