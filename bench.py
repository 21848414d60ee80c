#!/usr/bin/env python3
"""Headline benchmark: Chebyshev-K fwd+bwd samples/s on MI355X (BASELINE.json).

Workload (BASELINE.json configs[1]): MNIST 8-NN grid
graph coarsened to M=976 vertices (nnz(L~)=6396), K=25, Fin=1, Fout=32,
batch 256 per GPU, fp32.  One step = one training step of the chebyshev5
filter on synthetic data already resident in HBM:
    forward  (basis + y = basis W)          -> cg_cheb_forward
    backward (dx, dW) with a fixed N(0,1) upstream gradient dy -> cg_cheb_backward
    all-reduce(sum) of dW over ranks (RCCL), N>1 only
    Adam update of W (TF-1.x rule, grad scaled by 1/world)   -> cg_adam_update
Weak scaling: every rank processes its own batch of 256.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W]
        (N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)
Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import scipy.sparse
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from cnn_graph_amd import dist as cdist  # noqa: E402
from cnn_graph_amd import ops  # noqa: E402
from cnn_graph_amd.graph_conv import truncated_normal_  # noqa: E402
from cnn_graph_amd.plan import ChebPlan  # noqa: E402

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
MFMA_F32_PEAK_TF = 157.3   # dense fp32 MFMA


def load_config_b():
    """The M=976 coarsened MNIST graph produced by the reference recipe
    (tests/golden/make_golden.py::config_b); L is the normalized Laplacian."""
    with np.load(os.path.join(ROOT, "tests", "golden", "golden_B.npz"), allow_pickle=False) as z:
        L = scipy.sparse.csr_matrix((z["L_data"], z["L_indices"], z["L_indptr"]), shape=tuple(z["L_shape"]))
        fake = z["fake_rows"].copy()
    return L, fake


def algorithmic_bytes(M, nnz, B, K):
    """SURVEY.md §8d per-launch algorithmic bytes of the K-step SpMM basis."""
    csr = 8 * nnz + 4 * (M + 1)
    fwd = (K - 1) * csr + 4 * M * B * (2 + 3 * (K - 2))
    bwd = (K - 1) * csr + 4 * M * B * (3 + 5 * (K - 2))
    return fwd, bwd, csr


def cpu_baseline(L, fake, K, Fout, seconds=12.0, threads=16):
    """The oracle (tests-only CPU restatement, scipy SpMM + numpy GEMM) timed on
    a bounded sample of the same workload: batches of 32 samples, fwd+bwd."""
    from threadpoolctl import threadpool_limits
    from oracle import cheb_oracle as O
    from cnn_graph_amd.graph import rescale_L, canonical_csr
    rp, ci, v = canonical_csr(rescale_L(L, 2))
    M = L.shape[0]
    n = 32
    rng = np.random.default_rng(1)
    x = rng.random((n, M, 1), dtype=np.float32)
    x[:, fake, :] = 0
    W = (rng.standard_normal((K, Fout)) * 0.1).astype(np.float32)
    dy = rng.standard_normal((n, M, Fout)).astype(np.float32)
    with threadpool_limits(limits=threads):
        t0 = time.perf_counter()
        reps = 0
        while True:
            basis, _y = O.cheb_forward(x, rp, ci, v, W, K, dtype=np.float32)
            O.cheb_backward(dy, basis, W, rp, ci, v, n, M, 1, K, dtype=np.float32)
            reps += 1
            el = time.perf_counter() - t0
            if el > seconds:
                break
    return {"value": round(reps * n / el, 1), "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"{reps} fwd+bwd passes of a 32-sample batch of config B (oracle/cheb_oracle.py, "
                      f"fp32, scipy SpMM + numpy BLAS, {threads} BLAS threads), {el:.1f}s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=256, help="samples per GPU")
    ap.add_argument("--path", default="auto", choices=["auto", "resident", "stream"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    args = ap.parse_args()

    rank, world, local = cdist.init()
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    K, Fin, Fout = 25, 1, 32
    L, fake = load_config_b()
    M = L.shape[0]
    N = args.batch
    plan = ChebPlan.from_laplacian(L, lmax=2, device=local, path=args.path)
    path = plan.query_path(N, Fin, K, Fout)

    g = torch.Generator(device=dev)
    g.manual_seed(2017 + rank)
    x = torch.rand((N, M, Fin), device=dev, generator=g)
    x[:, torch.as_tensor(fake, device=dev, dtype=torch.long), :] = 0
    W = truncated_normal_(torch.empty((Fin * K, Fout), device=dev), 0.1)
    cdist.broadcast_parameters([W])
    dy = torch.randn((N, M, Fout), device=dev, generator=g)
    m_adam = torch.zeros_like(W)
    v_adam = torch.zeros_like(W)

    runner = ops.ChebRunner(plan, N, Fin, K, Fout, dev)
    ev = {k: [] for k in ("fwd", "bwd")}

    def step(i, timed):
        if timed:
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            e0.record()
        runner.forward(x, W)
        if timed:
            e1.record()
        _dx, dW = runner.backward(dy, W)
        if timed:
            e2.record()
            ev["fwd"].append((e0, e1))
            ev["bwd"].append((e1, e2))
        if world > 1:
            dist.all_reduce(dW, op=dist.ReduceOp.SUM)
        ops.adam_update(W, dW, m_adam, v_adam, i + 1, lr=1e-3, grad_scale=1.0 / world)

    for i in range(args.warmup):
        step(i, False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i, True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    fwd_ms = float(np.mean([a.elapsed_time(b) for a, b in ev["fwd"]]))
    bwd_ms = float(np.mean([a.elapsed_time(b) for a, b in ev["bwd"]]))
    B = N * Fin
    bytes_fwd, bytes_bwd, _csr = algorithmic_bytes(M, plan.nnz, B, K)
    compulsory_fwd = 4 * (N * M * Fin + N * M * Fin * K + N * M * Fout) + 8 * plan.nnz + 4 * (M + 1)
    kern = {
        "fwd": {"ms": fwd_ms, "alg_bytes": bytes_fwd},
        "bwd": {"ms": bwd_ms, "alg_bytes": bytes_bwd},
    }
    dom = max(kern, key=lambda k: kern[k]["ms"])
    ach = kern[dom]["alg_bytes"] / (kern[dom]["ms"] * 1e-3) / 1e9

    value = N * world * args.steps / elapsed
    out = {
        "metric": "Chebyshev-K fwd+bwd samples/sec",
        "value": round(value, 1),
        "unit": "samples/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (x~U[0,1) with fake vertices 0, dy~N(0,1), W~truncnorm(0,0.1)); "
                "graph = reference MNIST recipe M=976",
        "config": {"workload": "config B: MNIST 8-NN grid coarsened, M=976, nnz=6396, K=25, Fin=1, "
                               "Fout=32, chebyshev5 fwd+bwd + dW all-reduce + Adam",
                   "batch_per_gpu": N, "global_batch": N * world, "M": M, "nnz": plan.nnz, "K": K,
                   "Fin": Fin, "Fout": Fout, "path": path, "parallelism": f"dp{world}"},
        "roofline": {"bound": "hbm", "kernel": "cheb_fwd_resident" if dom == "fwd" and path == "resident"
                     else ("cheb_bwd_resident" if path == "resident" else f"stream_{dom}"),
                     "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None,
                     "alg_bytes_per_launch": kern[dom]["alg_bytes"],
                     "avg_launch_ms": round(kern[dom]["ms"], 5)},
        "kernels": {k: {"avg_ms": round(v["ms"], 5), "alg_bytes": v["alg_bytes"],
                        "alg_GBps": round(v["alg_bytes"] / (v["ms"] * 1e-3) / 1e9, 1)}
                    for k, v in kern.items()},
        "compulsory_fwd_bytes": compulsory_fwd,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(L, fake, K, Fout, seconds=args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
