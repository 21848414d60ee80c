#!/usr/bin/env python3
"""Step-schedule study on one GPU (config B, N=256): what the data-parallel
exchange would cost in each backward schedule, measured with a 1-rank RCCL
communicator (the all-reduce itself is then a local copy; what is measured is
the schedule's own cost: launches, cross-stream events, split dW).

  fused      fwd | bwd(dx + fused dW + slab reduce) | [allreduce] | adam     (bench.py)
  split      fwd | dW (weight_grad) | bwd(dx only) | [allreduce] | adam      (one stream)
  overlap    fwd | side: dW -> allreduce  ||  main: bwd(dx only) | join | adam
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from cnn_graph_amd import _lib, ops  # noqa: E402
from cnn_graph_amd.dist import RcclComm  # noqa: E402
from cnn_graph_amd.plan import ChebPlan  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    L, fake = bench.load_config_b()
    K, Fin, Fout, N = 25, 1, 32, 256
    plan = ChebPlan.from_laplacian(L, 2, 0)
    M = plan.M
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    x = torch.rand((N, M, Fin), device=dev, generator=g)
    W = torch.randn((Fin * K, Fout), device=dev, generator=g) * 0.1
    dy = torch.randn((N, M, Fout), device=dev, generator=g)
    m = torch.zeros_like(W)
    v = torch.zeros_like(W)
    r = ops.ChebRunner(plan, N, Fin, K, Fout, dev)
    comm = RcclComm(0)
    lib = _lib.lib()
    main_s = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev)
    ev_fork, ev_join = torch.cuda.Event(), torch.cuda.Event()
    dW2 = torch.empty_like(W)
    nb = ctypes.c_size_t()
    lib.cg_weight_grad_workspace_bytes(N * M, Fin * K, Fout, ctypes.byref(nb))
    wgws = torch.empty(nb.value, device=dev, dtype=torch.uint8)
    ms = main_s.cuda_stream
    ss = side.cuda_stream

    def adam(i, grad):
        lib.cg_adam_update(W.data_ptr(), grad.data_ptr(), m.data_ptr(), v.data_ptr(), W.numel(),
                           ctypes.c_float(1e-3), ctypes.c_float(0.9), ctypes.c_float(0.999),
                           ctypes.c_float(1e-8), i + 1, ctypes.c_float(1.0), ms)

    def fused(i, ar):
        r.forward(x, W, stream=ms)
        r.backward(dy, W, stream=ms)
        if ar:
            comm.allreduce_sum_(r.dW, ms)
        adam(i, r.dW)

    def split(i, ar):
        r.forward(x, W, stream=ms)
        lib.cg_weight_grad(N * M, Fin * K, Fout, r.basis.data_ptr(), dy.data_ptr(), dW2.data_ptr(),
                           0, wgws.data_ptr(), nb.value, ms)
        lib.cg_cheb_backward(plan.handle, N, Fin, K, Fout, dy.data_ptr(), r.basis.data_ptr(),
                             W.data_ptr(), r.dx.data_ptr(), None, r.bws.data_ptr(), r.bwd_bytes, ms)
        if ar:
            comm.allreduce_sum_(dW2, ms)
        adam(i, dW2)

    def overlap(i, ar):
        r.forward(x, W, stream=ms)
        ev_fork.record(main_s)
        side.wait_event(ev_fork)
        lib.cg_weight_grad(N * M, Fin * K, Fout, r.basis.data_ptr(), dy.data_ptr(), dW2.data_ptr(),
                           0, wgws.data_ptr(), nb.value, ss)
        if ar:
            comm.allreduce_sum_(dW2, ss)
        lib.cg_cheb_backward(plan.handle, N, Fin, K, Fout, dy.data_ptr(), r.basis.data_ptr(),
                             W.data_ptr(), r.dx.data_ptr(), None, r.bws.data_ptr(), r.bwd_bytes, ms)
        ev_join.record(side)
        main_s.wait_event(ev_join)
        adam(i, dW2)

    res = {}
    for name, fn in (("fused", fused), ("split", split), ("overlap", overlap)):
        for ar in (False, True):
            for i in range(20):
                fn(i, ar)
            torch.cuda.synchronize()
            vals = []
            for rep in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(main_s)
                for i in range(100):
                    fn(i, ar)
                e1.record(main_s)
                torch.cuda.synchronize()
                vals.append(e0.elapsed_time(e1) * 10)  # us per step
            res[f"{name}{'+ar' if ar else ''}"] = round(float(np.median(vals)), 2)
    print(json.dumps({"us_per_step": res}))
    comm.close()


if __name__ == "__main__":
    main()
