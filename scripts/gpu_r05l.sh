#!/bin/bash
# LSTM + dW + glstm DP tests, config E timing / kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05l}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lstm.py tests/test_gpu_dw_direct.py tests/test_gpu_glstm_dp.py > $OUT/pytest.txt 2>&1 || { echo TEST_FAIL; tail -60 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
timeout -k 10 300 python scripts/bench_configs.py E E --no-cpu > $OUT/E.jsonl 2>&1 || { echo E_FAIL; tail -20 $OUT/E.jsonl; exit 1; }
cat $OUT/E.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o E --output-format csv -- python3 scripts/bench_configs.py E --no-cpu > $OUT/kt.log 2>&1 || { echo KT_FAIL; tail -20 $OUT/kt.log; exit 1; }
find $OUT/kt -name "*kernel_stats.csv" -exec head -14 {} \;
