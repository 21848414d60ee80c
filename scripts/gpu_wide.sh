#!/bin/bash
# Streaming paths (configs C1/C2/D): parity tests, timing, and a rocprofv3
# kernel trace of C1 and C2.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-wide}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_parity.py tests/test_gpu_model.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
timeout -k 10 300 python scripts/bench_configs.py C1 C2 D > $OUT/cfg.jsonl 2>&1 || { tail -20 $OUT/cfg.jsonl; exit 1; }
grep config $OUT/cfg.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o kt --output-format csv -- python3 scripts/bench_configs.py C1 C2 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cut -c1-150 {} \; | head -16
