import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


def ensure_built():
    """Build libcheb_mi355.so in-tree if it is missing (hipcc cross-compiles
    gfx950 without a GPU)."""
    lib = os.path.join(ROOT, "cnn_graph_amd", "libcheb_mi355.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-C", ROOT, "-j8"], check=True, stdout=subprocess.DEVNULL)
    return lib


@pytest.fixture(scope="session")
def built_lib():
    return ensure_built()


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def case(g, prefix=""):
    """One filter case from a golden dict (keys optionally prefixed)."""
    d = {k[len(prefix):]: v for k, v in g.items() if k.startswith(prefix)}
    for k in ("M", "N", "Fin", "K", "Fout"):
        d[k] = int(d[k])
    return d


CASES = [("golden_A.npz", ""), ("golden_A.npz", "fin3_"), ("golden_A.npz", "k1_"),
         ("golden_A.npz", "k2_"), ("golden_B.npz", ""), ("golden_E.npz", "")]
CASE_IDS = ["A", "A_fin3", "A_k1", "A_k2", "B", "E"]


@pytest.fixture(scope="session")
def golden():
    cache = {}

    def get(name):
        if name not in cache:
            cache[name] = load_golden(name)
        return cache[name]
    return get


@pytest.fixture
def cg_opts():
    """Set kernel-selection options (cg_set_option) for one test:
    ``cg_opts("dw_direct", 0)``; every option touched is restored afterwards."""
    from cnn_graph_amd import _lib
    saved = {}

    def setter(name, value):
        prev = _lib.set_option(name, int(value))
        saved.setdefault(name, prev)
    yield setter
    for name, prev in saved.items():
        _lib.set_option(name, prev)
