"""Scratch timing of the dW GEMMs (CG_LIB_PATH selects the library): config E's
one-pass LSTM weight gradients, config D's planes dW at N = 32 and config C2's
rows dW, each with dw_x3 = 0 and 1; event-timed medians in ms."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cnn_graph_amd import _lib, ops  # noqa: E402


def med(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ts.sort()
    return round(ts[len(ts) // 2], 4)


dev = torch.device("cuda", 0)
g = torch.Generator(device=dev)
g.manual_seed(1)
out = {"lib": os.path.basename(os.environ.get("CG_LIB_PATH", "libcheb_mi355.so"))}
R, H, Fin, K = 12 * 128 * 1024, 32, 2, 3
hst, xst = R * H + 96, R * Fin + 40
hbuf = torch.randn((K * hst,), device=dev, generator=g)
xbuf = torch.randn((K * xst,), device=dev, generator=g)
dpre = torch.randn((R, 4 * H), device=dev, generator=g)
hpl, xpl = hbuf[:R * H].view(R, H), xbuf[:R * Fin].view(R, Fin)
for m in (0, 1):
    _lib.set_option("dw_x3", m)
    out[f"E_x3{m}"] = med(lambda: ops.lstm_weight_grads(hpl, hst, xpl, xst, K, R, dpre))
del hbuf, xbuf, dpre
R, Fin, K, Fo = 32 * 262144, 64, 3, 64
st = R * Fin
buf = torch.rand((K * st,), device=dev, generator=g)
D = torch.randn((R, Fo), device=dev, generator=g)
for m in (0, 1):
    _lib.set_option("dw_x3", m)
    out[f"D_x3{m}"] = med(lambda: ops.weight_grad_planes(buf[:st].view(R, Fin), st, K, R, D), 5)
del buf, D
R, FK, Fo = 128 * 10000, 160, 32
A = torch.randn((R, FK), device=dev, generator=g)
D = torch.randn((R, Fo), device=dev, generator=g)
for m in (0, 1):
    _lib.set_option("dw_x3", m)
    out[f"C2_x3{m}"] = med(lambda: ops.weight_grad(A, D))
print(json.dumps(out))
