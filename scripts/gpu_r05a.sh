#!/bin/bash
# Round-5 first GPU pass: the new tests first, then every -m gpu test, smoke,
# the bench line, C2 / D with x in plane 0 and a kernel trace of C2 / D.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05a}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_optim.py tests/test_gpu_glstm_dp.py tests/test_gpu_basis_layout.py tests/test_gpu_dp_bench.py > $OUT/pytest_new.txt 2>&1 || { echo NEW_FAIL; tail -60 $OUT/pytest_new.txt; exit 1; }
tail -1 $OUT/pytest_new.txt
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.txt; exit 1; }
tail -1 $OUT/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo SMOKE_FAIL; tail -30 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 5 > $OUT/bench.json 2>&1 || { echo BENCH_FAIL; tail -30 $OUT/bench.json; exit 1; }
tail -1 $OUT/bench.json
timeout -k 10 400 python scripts/bench_configs.py C2 D --d-batch 256 --no-cpu > $OUT/cfg.jsonl 2>&1 || { echo CFG_FAIL; tail -20 $OUT/cfg.jsonl; exit 1; }
grep config $OUT/cfg.jsonl
timeout -k 10 400 python scripts/bench_configs.py C2 D --d-batch 256 --no-cpu --copy-x > $OUT/cfg_copy.jsonl 2>&1 || { echo CFG2_FAIL; tail -20 $OUT/cfg_copy.jsonl; exit 1; }
grep config $OUT/cfg_copy.jsonl
