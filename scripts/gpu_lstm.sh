#!/bin/bash
# gconv-LSTM (config E): GPU tests, timing of the fused vs unfused h-step, and
# a rocprofv3 kernel trace of the fused layer.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-lstm}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_lstm.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
timeout -k 10 300 python scripts/bench_configs.py E E_unfused > $OUT/cfg.jsonl 2>&1 || { tail -20 $OUT/cfg.jsonl; exit 1; }
grep config $OUT/cfg.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o kt --output-format csv -- python3 scripts/bench_configs.py E > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cut -c1-150 {} \; | head -14
