#!/bin/bash
# rowgemm grid sizing: every -m gpu test, then C2 / D (N = 256) timing + D kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05o}
mkdir -p $OUT
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.txt; exit 1; }
tail -1 $OUT/pytest_gpu.txt
timeout -k 10 300 python scripts/bench_configs.py C2 --no-cpu > $OUT/C2.jsonl 2>&1 || { echo C2_FAIL; tail -20 $OUT/C2.jsonl; exit 1; }
grep config $OUT/C2.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ktD -o D --output-format csv -- python3 scripts/bench_configs.py D --d-batch 256 --no-cpu --rounds 1 > $OUT/D.log 2>&1 || { echo D_FAIL; tail -20 $OUT/D.log; exit 1; }
grep config $OUT/D.log
find $OUT/ktD -name "*kernel_stats.csv" -exec head -8 {} \;
