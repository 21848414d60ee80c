#!/usr/bin/env python3
"""Timing of the non-headline configurations of SURVEY.md §8d on one GPU
(bench.py measures the headline config B).  One JSON line per config:

  C1  20NEWS-like 10k-vertex graph, layer 1: N=128, Fin=1, K=5, Fout=32
  C2  same graph, layer 2:                  N=128, Fin=32, K=5, Fout=32
  D   Chung-Lu 2^18 vertices, nnz 4.19M:    N=--d-batch (default 32), Fin=Fout=64, K=3
  E   gconv-LSTM layer on grid(32) 8-NN:    T=12, N=128, Fin=2, H=32, K=3 (fwd+bwd, BPTT)

fwd / bwd are HIP-event timings (torch's current stream, where every C-ABI
call is enqueued) of one chebyshev5 forward and backward (dx + dW), median of
rounds; alg_GBps uses SURVEY.md §8d's algorithmic bytes.  Each line carries a
`cpu_baseline`: the oracle's fwd+bwd of the same config on the host cores
(bench.py's CPU legs -- the only place outside tests/ that runs oracle/),
median of the timed passes, with the sub-batch and pass count stated.
Usage: python scripts/bench_configs.py [A C1 C2 D E R] [--d-batch N] [--layout auto|rows|planes]
                                       [--no-cpu] [--cpu-seconds S]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import scipy.sparse
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))

import bench  # noqa: E402  (the CPU legs)
from cnn_graph_amd import ops  # noqa: E402
from cnn_graph_amd.plan import ChebPlan  # noqa: E402


ROUNDS = 3


def ev_ms(fn, reps=5, rounds=None):
    rounds = ROUNDS if rounds is None else rounds
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


def alg_bytes(M, nnz, B, K):
    csr = 8 * nnz + 4 * (M + 1)
    return (K - 1) * csr + 4 * M * B * (2 + 3 * (K - 2)), (K - 1) * csr + 4 * M * B * (3 + 5 * (K - 2))


def filter_config(name, Lt, N, Fin, K, Fout, dev, variant="auto", layout="auto", copy_x=False):
    M = Lt.shape[0]
    plan = ChebPlan(Lt, device=0, variant=variant)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    x = torch.rand((N, M, Fin), device=dev, generator=g)
    W = torch.randn((Fin * K, Fout), device=dev, generator=g) * 0.1
    dy = torch.randn((N, M, Fout), device=dev, generator=g)
    if layout == "auto":  # what the autograd layers use (ops.basis_layout_for)
        layout = ops.basis_layout_for(plan, N, Fin, K, Fout)
    if layout != "rows" and plan.basis_elems(N, Fin, K, Fout, layout) is None:
        return None  # the layout does not apply to this shape
    r = ops.ChebRunner(plan, N, Fin, K, Fout, dev, basis_layout=layout)
    x_in = "separate buffer (copied into plane 0)" if layout == "planes" else "separate buffer"
    if layout == "planes" and not copy_x:  # the input lives in plane 0: no copy of x
        r.input_plane().copy_(x)
        x = r.input_plane()
        x_in = "plane 0 of the basis (T_0 read in place)"
    r.forward(x, W)
    r.backward(dy, W)
    torch.cuda.synchronize()
    reps = 5 if M * N * Fin > 1e8 else 20
    f = ev_ms(lambda: r.forward(x, W), reps)
    b = ev_ms(lambda: r.backward(dy, W), reps)
    bf, bb = alg_bytes(M, plan.nnz, N * Fin, K)
    return {"config": name, "M": M, "nnz": plan.nnz, "N": N, "Fin": Fin, "K": K, "Fout": Fout,
            "path": r.path, "variant": variant, "basis_layout": layout, "input": x_in,
            "fwd_ms": round(f, 4), "bwd_ms": round(b, 4),
            "samples_per_s": round(N / ((f + b) * 1e-3), 1),
            "fwd_alg_GBps": round(bf / (f * 1e-3) / 1e9, 1),
            "bwd_alg_GBps": round(bb / (b * 1e-3) / 1e9, 1)}


def graph_e():
    """config E's grid graph: (L~, L = L~ + I so that rescale_L(L, 2) = L~)."""
    with np.load(os.path.join(ROOT, "tests", "golden", "golden_E.npz"), allow_pickle=False) as z:
        M = int(z["M"])
        Lt = scipy.sparse.csr_matrix((z["Lt_val"], z["Lt_col"], z["Lt_rowptr"]), shape=(M, M))
    return Lt, (Lt + scipy.sparse.identity(M, dtype=np.float32, format="csr")).tocsr()


def lstm_config(dev, T=12, N=128, Fin=2, H=32, K=3, hconv="auto"):
    from cnn_graph_amd.gconv_lstm import GConvLSTMCell, layer
    with np.load(os.path.join(ROOT, "tests", "golden", "golden_E.npz"), allow_pickle=False) as z:
        M = int(z["M"])
        Lt = scipy.sparse.csr_matrix((z["Lt_val"], z["Lt_col"], z["Lt_rowptr"]), shape=(M, M))
    # L = L~ + I  (rescale_L(L, 2) = L - I gives back this L~)
    L = (Lt + scipy.sparse.identity(M, dtype=np.float32, format="csr")).tocsr()
    cell = GConvLSTMCell(H, laplacian=L, lmax=2, K=K, feat_in=Fin, device=dev, hconv=hconv)
    M = L.shape[0]
    g = torch.Generator(device=dev)
    g.manual_seed(2)
    xs = torch.rand((T, N, M, Fin), device=dev, generator=g)
    gh = torch.randn((T, N, M, H), device=dev, generator=g)

    def fwd():
        with torch.no_grad():
            layer(cell, xs)

    def fwdbwd():
        hs, _ = layer(cell, xs)
        hs.backward(gh)

    fwdbwd()
    torch.cuda.synchronize()
    f = ev_ms(fwd, 3)
    fb = ev_ms(fwdbwd, 3)
    return {"config": "E", "hconv": "seq" if cell.seq else "fused" if cell.fused else "unfused",
            "M": M, "T": T, "N": N, "Fin": Fin, "H": H, "K": K,
            "fwd_ms": round(f, 3), "fwd_bwd_ms": round(fb, 3),
            "samples_per_s": round(N / (fb * 1e-3), 1)}


def resgnn_config(dev, N=100, Fin=2, nfilter=32, K=20, nres=4):
    """ResGNN training step (§8f-1, lib/graph_model.py:246-310 with
    lib/graph_conv.py:305-330): the humanflow-ln-period shape (M = 1024,
    nfilter 32, 4 residual layers, K 20, batch 100) on config E's
    1024-vertex graph -- 2*nres + 2 = 10 chebyshev5 calls per forward, the
    hidden ones with Fin = Fout = 32 (streaming path)."""
    from cnn_graph_amd.model import ResGNN
    with np.load(os.path.join(ROOT, "tests", "golden", "golden_E.npz"), allow_pickle=False) as z:
        M = int(z["M"])
        Lt = scipy.sparse.csr_matrix((z["Lt_val"], z["Lt_col"], z["Lt_rowptr"]), shape=(M, M))
    L = (Lt + scipy.sparse.identity(M, dtype=np.float32, format="csr")).tocsr()
    model = ResGNN(L, N=N, Fin=Fin, nfilter=nfilter, K=K, nres_layer_count=nres, device=dev)
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    x = torch.rand((N, M, Fin), device=dev, generator=g)
    labels = torch.rand((N, M, 2), device=dev, generator=g)
    paths = sorted({model.plan.query_path(N, fi, K, fo) for fi, fo in
                    ((Fin, nfilter), (nfilter, nfilter), (nfilter, 2))})
    ms = ev_ms(lambda: model.train_step(x, labels), reps=5)
    return {"config": "R", "M": M, "N": N, "Fin": Fin, "nfilter": nfilter, "K": K,
            "nres_layer_count": nres, "filter_calls_per_step": 2 * nres + 2, "paths": paths,
            "step_ms": round(ms, 3), "samples_per_s": round(N / (ms * 1e-3), 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["C1", "C2", "D", "E"])
    ap.add_argument("--d-batch", type=int, default=32)
    ap.add_argument("--variant", default="auto", help="plan variant (auto / narrow / ...)")
    ap.add_argument("--layout", default="auto", choices=["auto", "rows", "planes"],
                    help="basis layout of the C1/C2/D filters (auto: the autograd layers' choice, "
                         "ops.basis_layout_for -- planes where it applies, else rows)")
    ap.add_argument("--rounds", type=int, default=3, help="timed rounds per measurement (median)")
    ap.add_argument("--opt", action="append", default=[],
                    help="kernel-selection option name=value (cg_set_option), e.g. dw_direct=3")
    ap.add_argument("--copy-x", action="store_true",
                    help="planes layout: keep x in its own buffer (the forward copies it into plane 0)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline legs")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    args = ap.parse_args()
    global ROUNDS
    ROUNDS = args.rounds
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from cnn_graph_amd import _lib
    for kv in args.opt:
        name, val = kv.split("=")
        _lib.set_option(name, int(val))
    from cnn_graph_amd.graph import rescale_L
    for name in args.configs:
        cpu = None
        if name == "A":  # the usage recipe's 4-NN graph, M = 100
            with np.load(os.path.join(ROOT, "tests", "golden", "golden_A.npz"), allow_pickle=False) as z:
                M = int(z["M"])
                Lt = scipy.sparse.csr_matrix((z["Lt_val"], z["Lt_col"], z["Lt_rowptr"]), shape=(M, M))
            out = filter_config("A", Lt, 32, 1, 5, 4, dev, args.variant, args.layout, args.copy_x)
            cpu = lambda: bench.cpu_baseline_filter("A", Lt, 32, 32, 1, 5, 4,  # noqa: E731
                                                    seconds=args.cpu_seconds)
        elif name in ("C1", "C2"):
            with np.load(os.path.join(ROOT, "tests", "golden", "golden_C.npz"), allow_pickle=False) as z:
                M = int(z["M"])
                Lt = scipy.sparse.csr_matrix((z["Lt_val"], z["Lt_col"], z["Lt_rowptr"]), shape=(M, M))
            Fin = 1 if name == "C1" else 32
            out = filter_config(name, Lt, 128, Fin, 5, 32, dev, args.variant, args.layout, args.copy_x)
            # the oracle's C2 pass is ~27 s at N = 128: a sub-batch of 8
            nc = 128 if name == "C1" else 8
            cpu = lambda: bench.cpu_baseline_filter(name, Lt, nc, 128, Fin, 5, 32,  # noqa: E731
                                                    seconds=args.cpu_seconds,
                                                    warmup=10 if nc == 128 else 2)
        elif name == "D":
            import synth_graphs
            Lt = rescale_L(synth_graphs.config_d_laplacian(), 2)
            out = filter_config("D", Lt, args.d_batch, 64, 3, 64, dev, args.variant, args.layout, args.copy_x)
            cpu = lambda: bench.cpu_baseline_filter("D", Lt, 1, args.d_batch, 64, 3, 64,  # noqa: E731
                                                    seconds=args.cpu_seconds, warmup=1,
                                                    min_passes=3)
        elif name == "E":
            out = lstm_config(dev)
            cpu = lambda: bench.cpu_baseline_lstm(graph_e()[0], 8, 128, 12, 2, 32, 3,  # noqa: E731
                                                  seconds=args.cpu_seconds)
        elif name == "E_unfused":
            out = lstm_config(dev, hconv="unfused")
        elif name == "E_step":
            out = lstm_config(dev, hconv="fused")
        elif name == "R":
            out = resgnn_config(dev)
            cpu = lambda: bench.cpu_baseline_resgnn(graph_e()[1], 2, 100, 2, 32, 20, 4,  # noqa: E731
                                                    seconds=args.cpu_seconds)
        else:
            raise SystemExit(f"unknown config {name}")
        if out is not None:
            if not args.no_cpu and cpu is not None:
                out["cpu_baseline"] = cpu()
            print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
