"""bench.py's N > 1 step schedule (cnn_graph_amd/dp_step.py) at world size 2
(the schedule the scaling runs time had never run with two ranks):
forward-applied Adam (cg_cheb_forward_adam, W / m / v double-buffered), the dW
all-reduce between backward and the next forward, grad_scale = 1/world, on
config B's graph (K = 25, Fout = 32, the orders basis layout of the bench).
Two ranks share this box's one GPU over gloo (dist.TorchComm) and train on the
halves of a fixed batch; one process runs the whole batch with the one-GPU
schedules (Adam fused into the dW reduction, and the separate Adam launch)
at grad_scale 1/2.  Bars: both replicas bitwise equal after every step, and
their weights within 1e-5 (normwise) of the full-batch runs' after 1, 2 and 3
steps (lib/graph_model.py:296-298 is where the exchange sits)."""
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
def test_bench_schedule_world2_matches_full_batch(dev, tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import dp_bench_worker as Wk
    out = tmp_path / "dpb.npz"
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "tests", "dp_bench_worker.py"), str(out)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    d = np.load(out)
    assert int(d["world"]) == 2
    assert np.array_equal(d["W"], d["W_r1"]), "replicas diverged"
    L, x, dy, W0 = Wk.problem()
    full_fused = Wk.run(x, dy, W0, L, dev, 1, None, "fused", grad_scale=0.5)
    full_unfused = Wk.run(x, dy, W0, L, dev, 1, None, "unfused", grad_scale=0.5)
    assert np.array_equal(full_fused, full_unfused)  # the fused update is k_adam's, bitwise
    for n in range(Wk.STEPS):
        assert not np.array_equal(d["W"][n], W0)
        err = O.normwise_err(d["W"][n], full_fused[n].astype(np.float64))
        assert err < 1e-5, (n + 1, err)
