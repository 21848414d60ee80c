#!/bin/bash
# Round-5 pass: every -m gpu test, config E timing + kernel trace, C1 / C2 / D timings
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05b}
mkdir -p $OUT
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo PYTEST_FAIL; tail -60 $OUT/pytest_gpu.txt; exit 1; }
tail -1 $OUT/pytest_gpu.txt
timeout -k 10 300 python scripts/bench_configs.py E E C1 C2 D --d-batch 256 --no-cpu > $OUT/cfg.jsonl 2>&1 || { echo CFG_FAIL; tail -20 $OUT/cfg.jsonl; exit 1; }
grep config $OUT/cfg.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ktE -o E --output-format csv -- python3 scripts/bench_configs.py E --no-cpu > $OUT/ktE.log 2>&1 || { echo KT_FAIL; tail -20 $OUT/ktE.log; exit 1; }
find $OUT/ktE -name "*kernel_stats.csv" -exec head -4 {} \; | cut -c1-160
timeout -k 10 300 python scripts/bench_configs.py D --d-batch 256 --no-cpu --opt dw_direct=3 > $OUT/D_dw3.jsonl 2>&1 || { echo D3_FAIL; tail -20 $OUT/D_dw3.jsonl; exit 1; }
grep config $OUT/D_dw3.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ktD -o D --output-format csv -- python3 scripts/bench_configs.py D --d-batch 256 --no-cpu --rounds 1 > $OUT/ktD.log 2>&1 || { echo KTD_FAIL; tail -20 $OUT/ktD.log; exit 1; }
find $OUT/ktD -name "*kernel_stats.csv" -exec head -8 {} \; | cut -c1-160
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ktD3 -o D --output-format csv -- python3 scripts/bench_configs.py D --d-batch 256 --no-cpu --rounds 1 --opt dw_direct=3 > $OUT/ktD3.log 2>&1 || { echo KTD3_FAIL; tail -20 $OUT/ktD3.log; exit 1; }
find $OUT/ktD3 -name "*kernel_stats.csv" -exec head -8 {} \; | cut -c1-160
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ktD4 -o D --output-format csv -- python3 scripts/bench_configs.py D --d-batch 256 --no-cpu --rounds 1 --opt dw_direct=4 > $OUT/ktD4.log 2>&1 || { echo KTD4_FAIL; tail -20 $OUT/ktD4.log; exit 1; }
find $OUT/ktD4 -name "*kernel_stats.csv" -exec head -8 {} \; | cut -c1-160
grep config $OUT/ktD4.log
