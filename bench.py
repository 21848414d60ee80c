#!/usr/bin/env python3
"""Headline benchmark: Chebyshev-K fwd+bwd samples/s on MI355X (BASELINE.json).

Workload (BASELINE.json configs[1]): MNIST 8-NN grid
graph coarsened to M=976 vertices (nnz(L~)=6396), K=25, Fin=1, Fout=32,
batch 256 per GPU, fp32.  One step = one training step of the chebyshev5
filter on synthetic data already resident in HBM:
    forward  (basis + y = basis W)                     -> cg_cheb_forward
    backward (dx, dW) with a fixed N(0,1) upstream dy   -> cg_cheb_backward
    all-reduce(sum) of dW over ranks (RCCL), N>1 only
    Adam update of W (TF-1.x rule, grad scaled by 1/world) -> cg_adam_update, or at
    one GPU (no exchange) fused into the dW reduction     -> cg_cheb_backward_adam
Weak scaling (default): every rank processes its own batch of 256 (the batch
dimension is sharded; L~ and W are replicated -- SURVEY.md §8e).  Strong
scaling: --global-batch G fixes the whole job's batch and shards it over the
ranks (lib/graph_model.py:296-298 is where the exchange sits in the reference).

The timed loop issues exactly those C-ABI calls on torch's current stream
(ctypes, pre-bound arguments, no per-step allocation or event), bracketed by
barrier + synchronize; the max over ranks is reported.  After it, each kernel
is timed alone in bursts of back-to-back launches with HIP events recorded on
the same stream (roofline.achieved; the same bursts also run once before the
warmup to lift the GPU out of its idle clocks); rocprofv3 summaries of the
same command live under profiles/ (scripts/prof_pmc.sh), whose PMC-measured HBM bytes of
the dominant kernel are reported as roofline.traffic when they match this
configuration.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--global-batch G]
  N > 1 under torchrun (python -m torch.distributed.run --nproc-per-node N ...
  bench.py --gpus N): one rank per GPU, WORLD_SIZE must equal N.  N > 1
  without torchrun: bench.py starts that torchrun itself as a child process
  (before anything touches the GPU) and exits with its status.
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import socket
import subprocess
import sys
import time

import numpy as np
import scipy.sparse
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from cnn_graph_amd import _lib  # noqa: E402
from cnn_graph_amd import dist as cdist  # noqa: E402
from cnn_graph_amd import ops  # noqa: E402
from cnn_graph_amd.dp_step import ChebTrainStep  # noqa: E402
from cnn_graph_amd.graph_conv import truncated_normal_  # noqa: E402
from cnn_graph_amd.plan import ChebPlan  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
MFMA_F32_PEAK_TF = 157.3   # dense fp32 MFMA (= fp32 vector peak)
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_latest.json")


def load_config_b():
    """The M=976 coarsened MNIST graph produced by the reference recipe
    (tests/golden/make_golden.py::config_b); L is the normalized Laplacian."""
    with np.load(os.path.join(ROOT, "tests", "golden", "golden_B.npz"), allow_pickle=False) as z:
        L = scipy.sparse.csr_matrix((z["L_data"], z["L_indices"], z["L_indptr"]), shape=tuple(z["L_shape"]))
        fake = z["fake_rows"].copy()
    return L, fake


def algorithmic_bytes(M, nnz, B, K):
    """SURVEY.md §8d per-launch algorithmic bytes of the K-step SpMM basis
    (forward) and of the reverse recurrence (backward); B = Fin * N_local."""
    csr = 8 * nnz + 4 * (M + 1)
    fwd = (K - 1) * csr + 4 * M * B * (2 + 3 * (K - 2))
    bwd = (K - 1) * csr + 4 * M * B * (3 + 5 * (K - 2))
    return fwd, bwd, csr


def host_cpus():
    """(usable CPUs, affinity CPUs, cgroup quota or None, os.cpu_count()): the
    CPUs this process may actually run on -- the box's CPU share, not the
    machine's core count that os.cpu_count() reports."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    usable = aff if quota is None else max(1, min(aff, int(math.floor(quota))))
    return usable, aff, quota, os.cpu_count()


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_pass_times(fn, warmup=10, min_passes=50, seconds=10.0, max_passes=100000):
    """SURVEY.md §8d's timing rule for the CPU leg: `warmup` untimed passes,
    then timed passes until at least `min_passes` AND about `seconds` have
    run (capped by max_passes).  Returns the per-pass times (s)."""
    for _ in range(warmup):
        fn()
    times = []
    t_end = time.perf_counter() + seconds
    while len(times) < max_passes and (len(times) < min_passes or time.perf_counter() < t_end):
        t0 = time.perf_counter()
        fn()
        times.append(time.perf_counter() - t0)
    return times


def cpu_baseline(L, fake, K, Fout, n=256, seconds=10.0, warmup=10, min_passes=50):
    """The oracle (tests-only CPU restatement: scipy SpMM in the reference's
    order + numpy/BLAS GEMMs and layout transposes, fp32) timed on the SAME
    workload as the GPU line -- config B, batch 256, fwd+bwd -- as §8d says:
    the median of >= 50 timed passes after 10 warm-up passes, BLAS on every
    CPU this process may use (the scipy SpMM itself is single-threaded, as TF's
    CPU SparseTensorDenseMatMul functor the survey describes)."""
    from threadpoolctl import threadpool_limits
    from oracle import cheb_oracle as O
    from cnn_graph_amd.graph import rescale_L, canonical_csr
    rp, ci, v = canonical_csr(rescale_L(L, 2))
    M = L.shape[0]
    threads, aff, quota, ncpu = host_cpus()
    rng = np.random.default_rng(1)
    x = rng.random((n, M, 1), dtype=np.float32)
    x[:, fake, :] = 0
    W = (rng.standard_normal((K, Fout)) * 0.1).astype(np.float32)
    dy = rng.standard_normal((n, M, Fout)).astype(np.float32)

    def one_pass():
        basis, _y = O.cheb_forward(x, rp, ci, v, W, K, dtype=np.float32)
        O.cheb_backward(dy, basis, W, rp, ci, v, n, M, 1, K, dtype=np.float32)

    with threadpool_limits(limits=threads):
        times = cpu_pass_times(one_pass, warmup, min_passes, seconds)
    med = float(np.median(times))
    q = "none" if quota is None else f"{quota:g}"
    return {"value": round(n / med, 1), "unit": "samples/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "pass_ms_median": round(med * 1e3, 2),
            "pass_ms_p10": round(float(np.percentile(times, 10)) * 1e3, 2),
            "pass_ms_p90": round(float(np.percentile(times, 90)) * 1e3, 2),
            "value_p10_p90": [round(n / float(np.percentile(times, 90)), 1),
                              round(n / float(np.percentile(times, 10)), 1)],
            "sample": f"median of {len(times)} timed fwd+bwd passes (after {warmup} warm-up) of the "
                      f"full config-B batch (N={n}, M={M}, K={K}, Fout={Fout}; oracle/cheb_oracle.py, "
                      f"fp32); BLAS threads = {threads} = the CPUs this process may use (affinity "
                      f"{aff}, cgroup quota {q}; os.cpu_count() = {ncpu} is the whole machine); "
                      f"scipy SpMM single-threaded"}


def _cpu_leg(name, fn, n, n_full, what, warmup, min_passes, seconds, per_sample=True):
    """Time `fn` (one fwd+bwd pass over n samples of config `name`) on the host
    cores by cpu_pass_times; samples/s from the median pass.  n < n_full: a
    stated sub-batch of the config's per-GPU batch (the oracle's cost is linear
    in the batch: every sample is filtered independently)."""
    from threadpoolctl import threadpool_limits
    threads, aff, quota, ncpu = host_cpus()
    with threadpool_limits(limits=threads):
        times = cpu_pass_times(fn, warmup, min_passes, seconds)
    med = float(np.median(times))
    q = "none" if quota is None else f"{quota:g}"
    exc = "" if len(times) >= 50 and warmup >= 10 else (
        f" (exception to §8d's >= 50 after 10: {len(times)} passes after {warmup} warm-up, bounded "
        f"to ~{seconds:g} s of CPU work per config)")
    sub = "" if n == n_full else f" on a sub-batch of {n} of the config's {n_full} samples per GPU"
    return {"value": round(n / med, 2), "unit": "samples/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "pass_ms_median": round(med * 1e3, 2),
            "pass_ms_p10": round(float(np.percentile(times, 10)) * 1e3, 2),
            "pass_ms_p90": round(float(np.percentile(times, 90)) * 1e3, 2),
            "sample": f"config {name}: median of {len(times)} timed fwd+bwd passes{sub}; {what}; BLAS "
                      f"threads = {threads} (affinity {aff}, cgroup quota {q}; os.cpu_count() = {ncpu})"
                      + exc}


def cpu_baseline_filter(name, Lt, n, n_full, Fin, K, Fout, seconds=10.0, warmup=10, min_passes=50):
    """chebyshev5 fwd+bwd of configs C1 / C2 / D on the oracle (fp32, the
    reference's operation order: lib/graph.py:241-258, lib/graph_conv.py:155-176)."""
    from oracle import cheb_oracle as O
    from cnn_graph_amd.graph import canonical_csr
    rp, ci, v = canonical_csr(Lt)
    M = Lt.shape[0]
    rng = np.random.default_rng(1)
    x = rng.random((n, M, Fin), dtype=np.float32)
    W = (rng.standard_normal((Fin * K, Fout)) * 0.1).astype(np.float32)
    dy = rng.standard_normal((n, M, Fout)).astype(np.float32)

    def one_pass():
        basis, _y = O.cheb_forward(x, rp, ci, v, W, K, dtype=np.float32)
        O.cheb_backward(dy, basis, W, rp, ci, v, n, M, Fin, K, dtype=np.float32)

    return _cpu_leg(name, one_pass, n, n_full,
                    f"oracle/cheb_oracle.py fp32, M={M}, nnz={len(ci)}, Fin={Fin}, K={K}, Fout={Fout}",
                    warmup, min_passes, seconds)


def cpu_baseline_lstm(Lt, n, n_full, T, Fin, H, K, seconds=10.0, warmup=2, min_passes=50):
    """Config E: one gconv-LSTM layer's T-step forward + BPTT on the oracle
    (float64 restatement of lib/gconv_lstm.py:77-221 under static_rnn)."""
    from oracle import lstm_oracle as LO
    from cnn_graph_amd.graph import canonical_csr
    rp, ci, v = canonical_csr(Lt)
    lap = (rp, ci, v.astype(np.float64))
    M = Lt.shape[0]
    rng = np.random.default_rng(2)
    xs = rng.random((T, n, M, Fin))
    p = [rng.uniform(-0.1, 0.1, (K * Fin, 4 * H)), rng.uniform(-0.1, 0.1, (K * H, 4 * H)),
         rng.uniform(-0.3, 0.3, 4 * H)]
    gh = rng.standard_normal((T, n, M, H))

    def one_pass():
        _, _, caches = LO.layer_forward(xs, p, lap, K, H)
        LO.layer_backward(gh, None, caches, p, lap, K, H)

    return _cpu_leg("E", one_pass, n, n_full,
                    f"oracle/lstm_oracle.py float64, T={T}, M={M}, Fin={Fin}, H={H}, K={K}",
                    warmup, min_passes, seconds)


def cpu_baseline_resgnn(L, n, n_full, Fin, F, K, R, seconds=10.0, warmup=2, min_passes=50):
    """Config R: one ResGNN training step (forward, MSE, backward, Adam) on the
    oracle (float64 restatement of lib/graph_conv.py:305-330 + lib/graph_model.py:246-310)."""
    from oracle import model_oracle as MO
    from cnn_graph_amd.graph import canonical_csr, rescale_L
    rp, ci, v = canonical_csr(rescale_L(L, 2))
    lap = (rp, ci, v.astype(np.float64))
    M = L.shape[0]
    rng = np.random.default_rng(3)
    x = rng.random((n, M, Fin))
    labels = rng.random((n, M, 2))
    Ws = [rng.standard_normal((fi * K, fo)) * 0.1
          for fi, fo in [(Fin, F)] + [(F, F)] * (2 * R) + [(F, 2)]]
    state = [(np.zeros_like(w), np.zeros_like(w)) for w in Ws]

    def one_pass():
        MO.train_step(x, labels, Ws, lap, K, R, state, 1, 1e-3)

    return _cpu_leg("R", one_pass, n, n_full,
                    f"oracle/model_oracle.py float64, M={M}, Fin={Fin}, nfilter={F}, K={K}, "
                    f"{R} residual layers", warmup, min_passes, seconds)


def burst_ms(fn, reps=50, rounds=5):
    """Median over rounds of the mean per-launch time of `reps` back-to-back
    launches, HIP events recorded on torch's current stream (the launch stream)."""
    vals = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        vals.append(e0.elapsed_time(e1) / reps)
    return float(np.median(vals))


def pmc_traffic(kernel, cfg):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary
    (scripts/prof_pmc.sh -> profiles/pmc_latest.json) if it was taken on this
    configuration: FETCH_SIZE x 2 (gfx950 correction for wide coalesced reads,
    MI355X_MICROARCH.md §HBM) + WRITE_SIZE, both KB -> bytes."""
    try:
        with open(PMC_FILE) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    if d.get("config") != cfg:
        return None, None
    c = d.get("counters", {}).get(kernel)
    if not c or "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
        return None, None
    return int(c["FETCH_SIZE"] * 1024 * 2 + c["WRITE_SIZE"] * 1024), d.get("source")


def pmc_mfma_busy(kernel, cfg):
    """Fraction of `kernel`'s duration its MFMA pipe is busy, from the committed
    PMC summary's SQ_VALU_MFMA_BUSY_CYCLES (summed over the chip's 1024 SIMDs,
    so / (1024 x 2.4 GHz) = busy us per SIMD) over the kernel-trace average of
    the same summary; None when the summary is for another configuration."""
    try:
        with open(PMC_FILE) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, None
    if d.get("config") != cfg:
        return None, None
    c = d.get("counters", {}).get(kernel, {})
    k = d.get("kernels", {}).get(kernel, {})
    if "SQ_VALU_MFMA_BUSY_CYCLES" not in c or not k.get("avg_us"):
        return None, None
    busy_us = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * 2.4e3)
    return round(busy_us / k["avg_us"], 4), d.get("source")


def max_over_ranks(vals, dev):
    """Element-wise MAX of host floats over the ranks (a device tensor on
    nccl = RCCL, a host tensor on gloo)."""
    on_dev = dist.get_backend() == "nccl"
    tt = torch.tensor(vals, dtype=torch.float64, device=dev if on_dev else "cpu")
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    return [float(v) for v in tt.tolist()]


def spawn_ranks(n):
    """Re-launch this command under torchrun with n ranks (one per GPU) as a
    CHILD process -- nothing here has touched the GPU -- and return its status."""
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def batch_split(args, rank, world):
    """(per-rank batch, whole-job batch, strong?) for --batch / --global-batch."""
    if args.global_batch is not None:
        lo, hi = cdist.shard(args.global_batch, rank, world)
        if hi - lo < 1:
            sys.exit(f"bench.py: global batch {args.global_batch} < {world} ranks")
        return hi - lo, args.global_batch, True
    return args.batch, args.batch * world, False


def make_exchange(args, world, local):
    """The gradient exchange of configs D / E: (comm object with allreduce_sum_
    and world, rccl_nranks or None).  RCCL (cg_allreduce_sum_f32 on the compute
    stream) by default; torch.distributed (gloo in the one-GPU world-2 test)
    with --allreduce torch."""
    if not (world > 1 or args.force_allreduce):
        return None, None
    if args.allreduce == "rccl":
        comm = cdist.RcclComm(local)
        n = comm.nranks()
        if n != world:
            sys.exit(f"bench.py: RCCL communicator spans {n} ranks, expected {world}")
        return comm, n
    return cdist.TorchComm(), None


def timed_region(step, steps, warmup, world, dev):
    """W untimed steps, then exactly K steps bracketed by barrier + synchronize
    on both sides; the max over ranks of the elapsed seconds."""
    for i in range(warmup):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(warmup + i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed, = max_over_ranks([elapsed], dev)
    return elapsed


def train_step_d(args, N, world, local, dev, comm, rank):
    """Config D's data-parallel chebyshev5 training step (BASELINE configs[3]):
    the seeded Chung-Lu graph (scripts/synth_graphs.py, M = 2^18, nnz(L~) =
    4 189 524), Fin = Fout = 64, K = 3, N samples per rank; forward, backward
    (dx, dW), the all-reduce of dW (192 x 64 floats = 48 KB) when there is an
    exchange, then cg_adam_update (the unfused schedule of dp_step: one
    12 288-float launch against a ~0.2 s step).  Returns (step fn, info dict)."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import synth_graphs
    from cnn_graph_amd.graph import rescale_L
    K, Fin, Fout = 3, 64, 64
    Lt = rescale_L(synth_graphs.config_d_laplacian(), 2)
    plan = ChebPlan(Lt, device=local)
    layout = ops.basis_layout_for(plan, N, Fin, K, Fout)
    runner = ops.ChebRunner(plan, N, Fin, K, Fout, dev, basis_layout=layout)
    g = torch.Generator(device=dev)
    g.manual_seed(2017 + rank)
    if layout == "planes":  # the input lives in plane 0 of the basis (T_0 read in place)
        x = runner.input_plane()
        x.copy_(torch.rand(x.shape, device=dev, generator=g))
    else:
        x = torch.rand((N, plan.M, Fin), device=dev, generator=g)
    W = truncated_normal_(torch.empty((Fin * K, Fout), device=dev), 0.1)
    cdist.broadcast_parameters([W])
    dy = torch.randn((N, plan.M, Fout), device=dev, generator=g)
    allreduce = None
    if comm is not None:
        def allreduce(s):
            comm.allreduce_sum_(runner.dW, s)
    trainer = ChebTrainStep(runner, x, dy, W, world=world, allreduce=allreduce, schedule="unfused")
    stream = torch.cuda.current_stream(dev).cuda_stream

    def step(i):
        trainer.step(i, stream)

    def kernels():
        fwd = burst_ms(lambda: runner.forward(x, trainer.W[0], stream=stream), reps=2, rounds=3)
        bwd = burst_ms(lambda: runner.backward(dy, trainer.W[0], stream=stream), reps=2, rounds=3)
        bf, bb, _ = algorithmic_bytes(plan.M, plan.nnz, N * Fin, K)
        return {"fwd": {"kernel": "stream_fwd (k_cheb_step x 2 + k_rowgemm)", "ms": fwd, "alg_bytes": bf},
                "bwd": {"kernel": "stream_bwd (k_clenshaw_step + dBasis/dW GEMMs)", "ms": bwd,
                        "alg_bytes": bb}}

    info = {"workload": "config D: seeded Chung-Lu power-law graph, M=262144, K=3, Fin=64, Fout=64, "
                        "chebyshev5 fwd+bwd" + (" + dW all-reduce" if comm is not None else "") + " + Adam",
            "M": plan.M, "nnz": plan.nnz, "K": K, "Fin": Fin, "Fout": Fout,
            "path": plan.query_path(N, Fin, K, Fout), "basis_layout": layout,
            "grad_bucket_bytes": 4 * Fin * K * Fout, "adam": "cg_adam_update"}
    cpu = lambda: cpu_baseline_filter("D", Lt, 1, N, Fin, K, Fout, seconds=args.cpu_seconds,  # noqa: E731
                                      warmup=1, min_passes=3)
    return step, info, kernels, cpu, "bytes"


def train_step_e(args, N, world, local, dev, comm, rank):
    """Config E's data-parallel gconv-LSTM training step (BASELINE configs[4]):
    gconv_lstm.GLSTMModel -- inference_glstm = glstm_layer (one GConvLSTMCell,
    T = 12, K = 3, Fin = 2, H = 32, DropoutWrapper keep_prob 0.8) + fc_layer
    (lib/gconv_lstm.py:271-281, :609-636) -- MSE, backward through time, ONE
    all-reduce of the flat gradient bucket (13 376 floats = 53.5 KB) when there
    is an exchange, then Adam, on config E's 1 024-vertex grid graph; N
    samples per rank."""
    from cnn_graph_amd.gconv_lstm import GLSTMModel
    T, Fin, H, K, Fout = 12, 2, 32, 3, 2
    with np.load(os.path.join(ROOT, "tests", "golden", "golden_E.npz"), allow_pickle=False) as z:
        M = int(z["M"])
        Lt = scipy.sparse.csr_matrix((z["Lt_val"], z["Lt_col"], z["Lt_rowptr"]), shape=(M, M))
    L = (Lt + scipy.sparse.identity(M, dtype=np.float32, format="csr")).tocsr()  # rescale_L(L, 2) = L~
    model = GLSTMModel(L, N, T, Fin, num_hidden=H, K=K, out_features=Fout, keep_prob=0.8,
                       device=dev, seed=2017, comm=comm)
    cdist.broadcast_parameters([model.flat])
    g = torch.Generator(device=dev)
    g.manual_seed(2017 + rank)
    x = torch.rand((N, M, Fin * T), device=dev, generator=g)   # [N, M, F*T] as the reference feeds it
    labels = torch.rand((N, M, Fout), device=dev, generator=g)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def step(i):
        model.train_step(x, labels, stream)

    def kernels():
        with torch.no_grad():
            fwd = burst_ms(lambda: model.forward(x), reps=5, rounds=3)
        # gate contractions of one forward: T steps x N samples x M rows x
        # (K*Fin + K*H) inputs x 4H gate columns, 2 flops each
        flops = 2.0 * T * N * M * (K * Fin + K * H) * 4 * H
        return {"fwd": {"kernel": "glstm_layer forward (k_xbasis + k_lstm_seq) + fc cheb_conv",
                        "ms": fwd, "alg_flops": flops}}

    info = {"workload": "config E: gconv-LSTM (GLSTMModel: glstm_layer + fc_layer), grid graph M=1024, "
                        "T=12, K=3, Fin=2, H=32, keep_prob 0.8, MSE + BPTT"
                        + (" + gradient all-reduce" if comm is not None else "") + " + Adam",
            "M": M, "T": T, "K": K, "Fin": Fin, "H": H, "Fout": Fout,
            "grad_bucket_bytes": 4 * model.flat.numel(), "adam": "cg_adam_update (flat buffer)"}
    cpu = lambda: cpu_baseline_lstm(Lt, 8, N, T, Fin, H, K, seconds=args.cpu_seconds)  # noqa: E731
    return step, info, kernels, cpu, "flops"


def run_config_de(args, rank, world, local, dev, json_fd):
    """--config D / E: the config's training step through the contract's timed
    region (barrier + synchronize both sides, max over ranks); one JSON line on
    rank 0 with n_gpus, batch_per_gpu, global_batch and rccl_nranks."""
    N, N_global, strong = batch_split(args, rank, world)
    comm, rccl_nranks = make_exchange(args, world, local)
    build = train_step_d if args.config == "D" else train_step_e
    step, info, kernels, cpu, bound = build(args, N, world, local, dev, comm, rank)
    try:
        elapsed = timed_region(step, args.steps, args.warmup, world, dev)
    except Exception:
        if isinstance(comm, cdist.RcclComm) and comm.async_error(abort=True):
            sys.exit(f"bench.py: RCCL asynchronous error on rank {rank}")
        raise
    kern = kernels()
    if bound == "bytes":
        dom = max(kern, key=lambda k: kern[k]["ms"])
        ach = kern[dom]["alg_bytes"] / (kern[dom]["ms"] * 1e-3) / 1e9
        roof = {"bound": "hbm", "kernel": kern[dom]["kernel"], "achieved": round(ach, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                "traffic": None, "alg_bytes_per_launch": kern[dom]["alg_bytes"],
                "avg_launch_ms": round(kern[dom]["ms"], 4),
                "timing": "HIP events on the launch stream around back-to-back calls"}
    else:
        k = kern["fwd"]
        ach = k["alg_flops"] / (k["ms"] * 1e-3) / 1e12
        roof = {"bound": "mfma", "kernel": k["kernel"], "achieved": round(ach, 2),
                "peak": MFMA_F32_PEAK_TF, "unit": "TFLOP/s", "frac": round(ach / MFMA_F32_PEAK_TF, 4),
                "traffic": None, "alg_flops_per_call": k["alg_flops"], "avg_call_ms": round(k["ms"], 4),
                "timing": "HIP events on the launch stream around back-to-back forward calls"}
    info.update({"batch_per_gpu": N, "global_batch": N_global, "parallelism": f"dp{world}",
                 "allreduce": (args.allreduce if comm is not None else None),
                 "dist_backend": (dist.get_backend() if world > 1 else None),
                 "control_plane": (dist.get_backend() if world > 1 else None),
                 "rccl_nranks": rccl_nranks, "launch": "eager C-ABI calls per step"})
    out = {"metric": "Chebyshev-K fwd+bwd samples/sec", "value": round(N_global * args.steps / elapsed, 2),
           "unit": "samples/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(elapsed / args.steps * 1e3, 4), "higher_is_better": True,
           "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": "f32",
           "data": "synthetic (seeded inputs / labels, truncated-normal weights)",
           "config": info, "roofline": roof,
           "kernels": {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                       for k, v in kern.items()}}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu()
    if rank == 0:
        ctypes.CDLL(None).fflush(None)
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if comm is not None:
        torch.cuda.synchronize()
        comm.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default B 200, D 10, E 50)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default B 20, D 2, E 5)")
    ap.add_argument("--config", default="B", choices=["B", "D", "E"],
                    help="B (default, the headline: BASELINE configs[1]); D: the 2^18-vertex "
                         "power-law graph, Fin = Fout = 64, K = 3, 256 per GPU (configs[3]: 2 048 "
                         "over 8); E: the gconv-LSTM model, T = 12, 128 per GPU (configs[4]: 512 "
                         "over 4).  D and E time their own training step (train_step_d / "
                         "train_step_e below) through the same torchrun / barrier / max-over-ranks path")
    ap.add_argument("--batch", type=int, default=None,
                    help="samples per GPU (weak scaling; default 256 for B and D, 128 for E)")
    ap.add_argument("--global-batch", type=int, default=None,
                    help="fixed whole-job batch sharded over the ranks (strong scaling)")
    ap.add_argument("--path", default="auto", choices=["auto", "resident", "stream"])
    ap.add_argument("--basis-layout", default="orders", choices=["rows", "orders"],
                    help="saved-basis layout (orders: fast kernels, Fin <= 2 only; the default: "
                         "0.8 %% more samples/s than rows over 5 alternating runs, profiles/r03_layout)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--allreduce", default="rccl", choices=["rccl", "torch"],
                    help="rccl: cg_allreduce_sum_f32 on the compute stream (default); "
                         "torch: dist.all_reduce (ProcessGroupNCCL, internal stream + events)")
    ap.add_argument("--unfused-adam", action="store_true",
                    help="separate cg_adam_update launch even with no exchange step (ablation)")
    ap.add_argument("--force-allreduce", action="store_true",
                    help="run the gradient exchange even at N=1 (1-rank RCCL; overhead study)")
    ap.add_argument("--graph", default="off", choices=["on", "off"],
                    help="capture the K timed steps into one HIP graph before the timed region and "
                         "replay it there (every kernel of every step still runs); measured 0-1 %% "
                         "slower than eager launches on config B (profiles/r03_graph), so off")
    ap.add_argument("--opt", action="append", default=[],
                    help="kernel-selection option name=value (cg_set_option) for A/B runs, "
                         "e.g. dw_direct=0; the defaults are the measured-faster kernels")
    ap.add_argument("--dist-backend", default="auto", choices=["auto", "gloo"],
                    help="test only: gloo runs the N > 1 entry path (torchrun, init, barrier, max over "
                         "ranks) with every rank on GPU local_rank mod the visible GPUs, e.g. two "
                         "ranks on a one-GPU box (needs --allreduce torch: RCCL refuses two ranks "
                         "on one device); auto = nccl (RCCL) whenever a GPU is visible")
    args = ap.parse_args()
    dflt = {"B": (200, 20, 256), "D": (10, 2, 256), "E": (50, 5, 128)}[args.config]
    args.steps = dflt[0] if args.steps is None else args.steps
    args.warmup = dflt[1] if args.warmup is None else args.warmup
    args.batch = dflt[2] if args.batch is None else args.batch
    if args.dist_backend == "gloo" and args.allreduce != "torch":
        sys.exit("bench.py: --dist-backend gloo needs --allreduce torch")

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    # ONE JSON line on stdout: whatever the libraries print there (RCCL's
    # version banner at communicator init goes to stdout) is sent to stderr,
    # and the result line is written to the saved stdout descriptor
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    if env_world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}")
    # control plane (barriers, the max over ranks, the weight broadcast, the
    # RCCL unique id) over gloo whenever the gradient exchange is the library's
    # own RCCL communicator (the default): a rank then holds ONE RCCL
    # communicator, not ProcessGroupNCCL's as well
    ctrl = "gloo" if (args.dist_backend == "gloo" or args.allreduce == "rccl") else None
    rank, world, local = cdist.init(ctrl)
    if args.dist_backend == "gloo":
        local %= torch.cuda.device_count()
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    for kv in args.opt:
        name, val = kv.split("=")
        _lib.set_option(name, int(val))
    if args.config != "B":
        run_config_de(args, rank, world, local, dev, json_fd)
        return

    K, Fin, Fout = 25, 1, 32
    L, fake = load_config_b()
    M = L.shape[0]
    strong = args.global_batch is not None
    if strong:
        lo, hi = cdist.shard(args.global_batch, rank, world)
        N = hi - lo
        if N < 1:
            sys.exit(f"bench.py: global batch {args.global_batch} < {world} ranks")
    else:
        N = args.batch
    N_global = args.global_batch if strong else N * world
    plan = ChebPlan.from_laplacian(L, lmax=2, device=local, path=args.path)
    path = plan.query_path(N, Fin, K, Fout)

    g = torch.Generator(device=dev)
    g.manual_seed(2017 + rank)
    x = torch.rand((N, M, Fin), device=dev, generator=g)
    x[:, torch.as_tensor(fake, device=dev, dtype=torch.long), :] = 0
    W = truncated_normal_(torch.empty((Fin * K, Fout), device=dev), 0.1)
    cdist.broadcast_parameters([W])
    dy = torch.randn((N, M, Fout), device=dev, generator=g)

    runner = ops.ChebRunner(plan, N, Fin, K, Fout, dev, basis_layout=args.basis_layout)
    stream = torch.cuda.current_stream(dev).cuda_stream
    exchange = world > 1 or args.force_allreduce
    comm = None
    rccl_nranks = None
    allreduce = None
    if exchange and args.allreduce == "rccl":
        comm = cdist.RcclComm(local)
        ar_fn = _lib.lib().cg_allreduce_sum_f32
        ar_args = (comm.handle, runner.dW.data_ptr(), runner.dW.numel())
        # proof that the timed exchange spans every rank (ncclCommCount)
        rccl_nranks = comm.nranks()
        if rccl_nranks != world:
            sys.exit(f"bench.py: RCCL communicator spans {rccl_nranks} ranks, expected {world}")

        def allreduce(s):
            st = ar_fn(*ar_args, s)
            if st:
                _lib.check("cg_allreduce_sum_f32", st)
    elif exchange:
        tcomm = cdist.TorchComm()  # ProcessGroupNCCL on RCCL, a host copy on gloo

        def allreduce(s):
            tcomm.allreduce_sum_(runner.dW)

    # The step schedule (cnn_graph_amd/dp_step.py, driven at world 2 by
    # tests/test_gpu_dp_bench.py): with no exchange step (one GPU) the Adam
    # update rides on the dW reduction (cg_cheb_backward_adam) instead of a
    # separate launch; with an exchange (N > 1) the update of the all-reduced dW
    # is applied by the NEXT step's forward (cg_cheb_forward_adam: W, m, v
    # double-buffered, no Adam launch), so every timed step is one forward,
    # backward, all-reduce and Adam update.
    trainer = ChebTrainStep(runner, x, dy, W, world=world, allreduce=allreduce,
                            schedule="unfused" if args.unfused_adam else "auto")
    fuse_adam, fwd_adam = trainer.schedule == "fused", trainer.schedule == "forward"

    def step(i, stream=stream):
        trainer.step(i, stream)

    # HIP graph of the K timed steps (captured untimed, after the warmup): the
    # timed region is one replay, so the host's per-launch cost (ctypes + the
    # HIP launch path, ~2 launches per step) no longer sits in front of the
    # first kernel or between steps.  Each step keeps its own Adam step count.
    use_graph = args.graph == "on" and not (exchange and args.allreduce == "torch")
    graph = None

    def check_comm():
        """After a failed step: poll RCCL's asynchronous error
        and abort the communicator so blocked ranks return."""
        if comm is not None:
            st = comm.async_error(abort=True)
            if st:
                sys.exit(f"bench.py: RCCL asynchronous error {st} on rank {rank}")

    # Before the warmup: ~12 ms of back-to-back forward / backward launches
    # (the per-kernel timing bursts below, results discarded) that bring the
    # GPU out of its idle clock state, which otherwise lasts through a short
    # timed region (driver's 20-step run: steps at 0.060 ms that settle at
    # 0.057 ms after ~200 steps, profiles/r03_graph).  They touch no training
    # state.  The kernel timings themselves are taken after the timed region.
    burst_ms(lambda: runner.forward(x, W, stream=stream))
    burst_ms(lambda: runner.backward(dy, W, stream=stream))

    try:
        for i in range(args.warmup):
            step(i)
        torch.cuda.synchronize()
        if use_graph:
            graph = torch.cuda.CUDAGraph()
            cap = torch.cuda.Stream(dev)
            cap.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.graph(graph, stream=cap):
                for i in range(args.steps):
                    step(args.warmup + i, stream=cap.cuda_stream)
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if graph is not None:
            graph.replay()
        else:
            for i in range(args.steps):
                step(args.warmup + i)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
    except Exception:
        check_comm()
        raise
    check_comm()
    if world > 1:
        elapsed, = max_over_ranks([elapsed], dev)

    # per-step distribution (SURVEY.md §8d asks for the median step): a second
    # pass of the same steps with a HIP event between consecutive steps on
    # the launch stream (after the contract's timed region, which stays
    # event-free); max over ranks of each rank's median
    nstep = max(50, min(args.steps, 400))
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(nstep + 1)]
    if world > 1:
        dist.barrier()
    evs[0].record()
    for i in range(nstep):
        step(args.warmup + args.steps + i)
        evs[i + 1].record()
    torch.cuda.synchronize()
    per_step = np.array([evs[i].elapsed_time(evs[i + 1]) for i in range(nstep)])
    med_ms = float(np.median(per_step))
    p90_ms = float(np.percentile(per_step, 90))
    if world > 1:
        med_ms, p90_ms = max_over_ranks([med_ms, p90_ms], dev)

    # per-kernel timing (roofline.achieved), on the warm GPU: forward = one
    # kernel; backward = the recurrence kernel + the tiny fixed-order dW slab reduce
    fwd_ms = burst_ms(lambda: runner.forward(x, W, stream=stream))
    bwd_ms = burst_ms(lambda: runner.backward(dy, W, stream=stream))
    B = N * Fin
    bytes_fwd, bytes_bwd, _csr = algorithmic_bytes(M, plan.nnz, B, K)
    compulsory_fwd = 4 * (N * M * Fin + N * M * Fin * K + N * M * Fout) + 8 * plan.nnz + 4 * (M + 1)
    fwd_kernel = "cheb_fwd_fast" if path == "resident" else "stream_fwd"
    bwd_kernel = "cheb_bwd_fast" if path == "resident" else "stream_bwd"
    kern = {
        "fwd": {"kernel": fwd_kernel, "ms": fwd_ms, "alg_bytes": bytes_fwd},
        "bwd": {"kernel": bwd_kernel + "+k_reduce_slabs", "ms": bwd_ms, "alg_bytes": bytes_bwd},
    }
    dom = max(kern, key=lambda k: kern[k]["ms"])
    ach = kern[dom]["alg_bytes"] / (kern[dom]["ms"] * 1e-3) / 1e9
    cfg_key = {"M": M, "N": N, "K": K, "Fin": Fin, "Fout": Fout, "layout": runner.basis_layout}
    traffic, traffic_src = pmc_traffic(kern[dom]["kernel"].split("+")[0], cfg_key)
    fwd_traffic, _ = pmc_traffic(fwd_kernel, cfg_key)
    mfma_busy, mfma_src = pmc_mfma_busy(fwd_kernel, cfg_key)
    contraction_tflops = 2.0 * N * M * Fin * K * Fout / (fwd_ms * 1e-3) / 1e12
    spmm_ach = bytes_fwd / (fwd_ms * 1e-3) / 1e9

    value = N_global * args.steps / elapsed
    out = {
        "metric": "Chebyshev-K fwd+bwd samples/sec",
        "value": round(value, 1),
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "step_ms_median": round(med_ms, 4),
        "step_ms_p90": round(p90_ms, 4),
        "samples_per_s_at_median": round(N_global / (med_ms * 1e-3), 1),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (x~U[0,1) with fake vertices 0, dy~N(0,1), W~truncnorm(0,0.1)); "
                "graph = reference MNIST recipe M=976",
        "config": {"workload": "config B: MNIST 8-NN grid coarsened, M=976, nnz=6396, K=25, Fin=1, "
                               "Fout=32, chebyshev5 fwd+bwd" + (" + dW all-reduce" if exchange else "")
                               + " + Adam",
                   "batch_per_gpu": N, "global_batch": N_global, "M": M, "nnz": plan.nnz, "K": K,
                   "Fin": Fin, "Fout": Fout, "path": path, "basis_layout": runner.basis_layout,
                   "parallelism": f"dp{world}",
                   "allreduce": (args.allreduce if exchange else None),
                   "dist_backend": (dist.get_backend() if world > 1 else None),
                   "control_plane": (dist.get_backend() if world > 1 else None),
                   "rccl_nranks": rccl_nranks,
                   "options": dict(kv.split("=") for kv in args.opt) or None,
                   "launch": ("one HIP graph replay of the K captured steps" if graph is not None
                              else "eager C-ABI calls per step"),
                   "adam": ("fused into the dW reduction (cg_cheb_backward_adam)" if fuse_adam
                            else "applied by the next step's forward (cg_cheb_forward_adam)"
                            if fwd_adam else "cg_adam_update")},
        "roofline": {"bound": "hbm", "kernel": kern[dom]["kernel"],
                     "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(ach / HBM_PEAK_GBS, 4),
                     "traffic": traffic,
                     "alg_bytes_per_launch": kern[dom]["alg_bytes"],
                     "avg_launch_ms": round(kern[dom]["ms"], 5),
                     "timing": "HIP events on the launch stream around 50 back-to-back launches",
                     "traffic_source": traffic_src},
        # BASELINE.json's north-star target: >= 40 % of the HBM roofline on the
        # K-step CSR SpMM of config B, i.e. the forward basis kernel (the
        # headline `roofline` above is the slowest kernel of the step)
        "roofline_spmm_fwd": {"bound": "hbm", "kernel": fwd_kernel, "achieved": round(spmm_ach, 1),
                              "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": round(spmm_ach / HBM_PEAK_GBS, 4), "target_frac": 0.40,
                              "traffic": fwd_traffic, "alg_bytes_per_launch": bytes_fwd,
                              "avg_launch_ms": round(fwd_ms, 5)},
        "kernels": {k: {"kernel": v["kernel"], "avg_ms": round(v["ms"], 5), "alg_bytes": v["alg_bytes"],
                        "alg_GBps": round(v["alg_bytes"] / (v["ms"] * 1e-3) / 1e9, 1)}
                    for k, v in kern.items()},
        "contraction_mfma": {"tflops_over_fwd_kernel": round(contraction_tflops, 2),
                             "peak_tflops": MFMA_F32_PEAK_TF,
                             "frac": round(contraction_tflops / MFMA_F32_PEAK_TF, 4),
                             "busy_frac": mfma_busy, "busy_source": mfma_src},
        "compulsory_fwd_bytes": compulsory_fwd,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(L, fake, K, Fout, seconds=args.cpu_seconds)
    if rank == 0:
        ctypes.CDLL(None).fflush(None)  # library stdio buffers: still to stderr
        os.write(json_fd, (json.dumps(out) + "\n").encode())
    if comm is not None:
        torch.cuda.synchronize()
        comm.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
