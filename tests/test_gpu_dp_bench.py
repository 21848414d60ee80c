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


def _bench_json(args, timeout=400):
    """Run bench.py as the driver does (no WORLD_SIZE: bench.py starts its own
    torchrun child) and return its one JSON line."""
    import json
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py")] + args
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0])


@pytest.mark.timeout(900)
def test_bench_entry_path_world2(dev):
    """bench.py's own N > 1 entry: spawn_ranks -> torchrun ->
    cdist.init -> barrier -> timed steps -> max over ranks -> one JSON line on
    rank 0, with two ranks sharing this box's GPU over gloo (--dist-backend gloo,
    test only; RCCL refuses two ranks on one device).  Weak scaling: 256 per GPU,
    512 in all; strong scaling (--global-batch 256): 128 per GPU."""
    base = ["--gpus", "2", "--allreduce", "torch", "--dist-backend", "gloo", "--steps", "20",
            "--warmup", "5"]
    weak = _bench_json(base)
    assert weak["n_gpus"] == 2 and weak["steps"] == 20 and weak["warmup"] == 5
    assert weak["scaling"] == "weak"
    c = weak["config"]
    assert c["parallelism"] == "dp2" and c["global_batch"] == 512 and c["batch_per_gpu"] == 256
    assert c["allreduce"] == "torch" and c["dist_backend"] == "gloo"
    assert c["adam"].startswith("applied by the next step's forward")
    assert weak["value"] > 0 and weak["ms_per_step"] > 0
    assert abs(weak["value"] - 512 * 20 / (weak["ms_per_step"] * 20 / 1e3)) < 0.01 * weak["value"]
    assert "cpu_baseline" not in weak  # rank 0 at N = 1 only
    strong = _bench_json(base + ["--global-batch", "256"])
    assert strong["scaling"] == "strong" and strong["n_gpus"] == 2
    assert strong["config"]["batch_per_gpu"] == 128 and strong["config"]["global_batch"] == 256
    assert strong["value"] > 0


@pytest.mark.timeout(900)
@pytest.mark.parametrize("config,batch,bucket", [("D", 2, 4 * 192 * 64), ("E", 4, 53504)])
def test_bench_config_de_entry_world2(dev, config, batch, bucket):
    """bench.py --config D / E (BASELINE configs[3] is an
    8-GPU D, configs[4] a 4-GPU E) through the same N > 1 entry as config B:
    spawn_ranks -> torchrun -> init -> barrier -> timed steps -> max over ranks
    -> one JSON line, two ranks on this box's GPU over gloo, a reduced
    per-rank batch (the full shapes otherwise).  Weak and strong scaling."""
    base = ["--config", config, "--gpus", "2", "--allreduce", "torch", "--dist-backend", "gloo",
            "--batch", str(batch), "--steps", "3", "--warmup", "1"]
    weak = _bench_json(base)
    assert weak["n_gpus"] == 2 and weak["steps"] == 3 and weak["warmup"] == 1
    assert weak["scaling"] == "weak" and weak["metric"] == "Chebyshev-K fwd+bwd samples/sec"
    c = weak["config"]
    assert c["workload"].startswith(f"config {config}:")
    assert c["parallelism"] == "dp2" and c["batch_per_gpu"] == batch and c["global_batch"] == 2 * batch
    assert c["allreduce"] == "torch" and c["dist_backend"] == "gloo" and c["rccl_nranks"] is None
    assert c["grad_bucket_bytes"] == bucket
    assert weak["value"] > 0 and weak["ms_per_step"] > 0
    assert abs(weak["value"] - 2 * batch * 3 / (weak["ms_per_step"] * 3 / 1e3)) < 0.01 * weak["value"]
    r = weak["roofline"]
    assert r["bound"] == ("hbm" if config == "D" else "mfma") and 0 < r["frac"] < 1
    assert "cpu_baseline" not in weak
    strong = _bench_json(base[:-6] + ["--global-batch", str(2 * batch - 1), "--steps", "2", "--warmup", "1"])
    assert strong["scaling"] == "strong" and strong["config"]["global_batch"] == 2 * batch - 1
    assert strong["config"]["batch_per_gpu"] == batch - 1  # rank 0's shard; rank 1 takes the remainder


@pytest.mark.timeout(600)
def test_bench_config_e_one_gpu_line(dev):
    """bench.py --config E at N = 1 (the 1-rank line, with its exchange forced
    through a 1-rank RCCL communicator: rccl_nranks == 1) and the contract
    fields."""
    line = _bench_json(["--config", "E", "--batch", "8", "--steps", "3", "--warmup", "1",
                        "--no-cpu-baseline", "--force-allreduce"])
    assert line["n_gpus"] == 1 and line["config"]["rccl_nranks"] == 1
    assert line["config"]["global_batch"] == 8 and line["config"]["parallelism"] == "dp1"
    assert line["roofline"]["unit"] == "TFLOP/s"
