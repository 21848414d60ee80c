"""The fast path's bank-aware LDS layout (cnn_graph_amd/csrc/lds_layout.cpp,
host code run at plan creation) on config B's graph, through the host model of
cheb_fwd_fast's LDS accesses (scripts/ldsmodel/lds_model.cpp: the bank rule of
MI355X_MICROARCH.md §LDS per 32-lane half).  The model reproduced the PMC
passes' SQ_LDS_BANK_CONFLICT per instruction group exactly
(profiles/r04_lds); the layout must keep the own-record writes, the gathers
and the MFMA tile reads conflict-free, and be a deterministic function of the
graph."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.fixture(scope="module")
def model(tmp_path_factory):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    d = tmp_path_factory.mktemp("ldsmodel")
    exe = str(d / "lds_model")
    src = os.path.join(ROOT, "scripts", "ldsmodel", "lds_model.cpp")
    lay = os.path.join(ROOT, "cnn_graph_amd", "csrc", "lds_layout.cpp")
    subprocess.run([HIPCC, "-O2", "-std=c++17", src, lay, "-o", exe], check=True,
                   capture_output=True, timeout=300)
    import scipy.sparse
    from cnn_graph_amd import graph as G
    with np.load(os.path.join(ROOT, "tests", "golden", "golden_B.npz"), allow_pickle=False) as z:
        L = scipy.sparse.csr_matrix((z["L_data"], z["L_indices"], z["L_indptr"]), shape=tuple(z["L_shape"]))
    Lt = G.rescale_L(L, 2).tocsr()
    np.array([Lt.shape[0]], np.int32).tofile(str(d / "M.bin"))
    Lt.indptr.astype(np.int32).tofile(str(d / "rp.bin"))
    Lt.indices.astype(np.int32).tofile(str(d / "ci.bin"))
    return exe, d


def run(model):
    exe, d = model
    out = subprocess.run([exe, str(d / "M.bin"), str(d / "rp.bin"), str(d / "ci.bin"), "25", "256"],
                         check=True, capture_output=True, text=True, timeout=120).stdout
    return json.loads(out)


def test_config_b_layout_conflict_free(model):
    r = run(model)
    assert r["M"] == 976
    assert r["gather_groups_per_step"] == 216
    assert r["dispatch_extra"] == {"gathers": 0, "writes": 0, "tiles": 0}


def test_layout_deterministic(model):
    assert run(model) == run(model)
