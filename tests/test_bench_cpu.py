"""The bench's measurement arithmetic (no GPU): SURVEY.md §8d's algorithmic
bytes for config B and the other BASELINE configs the survey quotes, the PMC
lookup keyed by configuration, and the command-line contract's defaults."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
bench = pytest.importorskip("bench")


def test_algorithmic_bytes_config_b():
    # B 72.28 MB forward; DESIGN.md §5: 119.25 MB backward
    fwd, bwd, csr = bench.algorithmic_bytes(976, 6396, 256 * 1, 25)
    assert csr == 8 * 6396 + 4 * 977
    assert fwd == 72280928
    assert bwd == 119253856


def test_algorithmic_bytes_survey_figures():
    # C layer 1 62.3 MB (M 10 000, nnz 182 466, N 128, Fin 1,
    # K 5); D per GPU 85.9 GB (M 2^18, nnz 4 189 524, N 256, Fin 64, K 3)
    c1, _, _ = bench.algorithmic_bytes(10000, 182466, 128, 5)
    assert abs(c1 / 1e6 - 62.3) < 0.1
    d, _, _ = bench.algorithmic_bytes(262144, 4189524, 256 * 64, 3)
    assert abs(d / 1e9 - 85.9) < 0.1


def test_pmc_lookup_matches_only_its_configuration(tmp_path, monkeypatch):
    cfg = {"M": 976, "N": 256, "K": 25, "Fin": 1, "Fout": 32, "layout": "orders"}
    # raw rocprofv3 units: FETCH_SIZE / WRITE_SIZE in KB (FETCH x 2 on gfx950),
    # SQ_VALU_MFMA_BUSY_CYCLES summed over 1024 SIMDs at 2.4 GHz
    pmc = {"config": cfg, "source": "test",
           "kernels": {"cheb_bwd_fast": {"avg_us": 10.0}},
           "counters": {"cheb_bwd_fast": {"FETCH_SIZE": 50.0, "WRITE_SIZE": 2.0,
                                          "SQ_VALU_MFMA_BUSY_CYCLES": 1024 * 2.4e3 * 2.5}}}
    f = tmp_path / "pmc.json"
    f.write_text(json.dumps(pmc))
    monkeypatch.setattr(bench, "PMC_FILE", str(f))
    traffic, src = bench.pmc_traffic("cheb_bwd_fast", cfg)
    assert traffic == (50 * 2 + 2) * 1024 and src == "test"
    other = dict(cfg, layout="rows")
    assert bench.pmc_traffic("cheb_bwd_fast", other)[0] is None
    assert bench.pmc_mfma_busy("cheb_bwd_fast", cfg)[0] == 0.25


def test_committed_pmc_summary_is_config_b():
    with open(os.path.join(ROOT, "profiles", "pmc_latest.json")) as fh:
        d = json.load(fh)
    assert d["config"] == {"M": 976, "N": 256, "K": 25, "Fin": 1, "Fout": 32, "layout": "orders"}
    assert d["counters"]["cheb_bwd_fast"]["FETCH_SIZE_x2_bytes"] > 0


def test_batch_split_weak_and_strong():
    import argparse
    weak = argparse.Namespace(batch=256, global_batch=None)
    assert bench.batch_split(weak, 3, 8) == (256, 2048, False)  # config D: 2 048 over 8
    strong = argparse.Namespace(batch=128, global_batch=512)
    assert bench.batch_split(strong, 0, 4) == (128, 512, True)  # config E: 512 over 4
    odd = argparse.Namespace(batch=1, global_batch=7)
    assert [bench.batch_split(odd, r, 2)[0] for r in range(2)] == [3, 4]
