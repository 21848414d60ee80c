#!/usr/bin/env python3
"""Config B's rescaled Laplacian pattern (the fast path's L~) as three int32
files for lds_model:  python3 scripts/ldsmodel/export_b.py OUTDIR
then  hipcc -O2 -std=c++17 scripts/ldsmodel/lds_model.cpp cnn_graph_amd/csrc/lds_layout.cpp -o lds_model
      ./lds_model OUTDIR/M.bin OUTDIR/rp.bin OUTDIR/ci.bin 25 256"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from cnn_graph_amd import graph as G  # noqa: E402

out = sys.argv[1] if len(sys.argv) > 1 else "/tmp"
L, _ = bench.load_config_b()
Lt = G.rescale_L(L, 2).tocsr()
np.array([Lt.shape[0]], np.int32).tofile(os.path.join(out, "M.bin"))
Lt.indptr.astype(np.int32).tofile(os.path.join(out, "rp.bin"))
Lt.indices.astype(np.int32).tofile(os.path.join(out, "ci.bin"))
print(Lt.shape, Lt.nnz)
