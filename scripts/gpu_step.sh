#!/bin/bash
# Scratch GPU step (rewritten per experiment): LSTM / dropout tests, then the
# config E bench and its kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-step}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_ops.py tests/test_gpu_lstm.py tests/test_gpu_glstm_dp.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1; rc=$?
tail -3 $OUT/pytest.txt; [ $rc = 0 ] || exit 1
for i in 1 2; do
timeout -k 10 300 python bench.py --config E --no-cpu-baseline > $OUT/E.$i.json 2>$OUT/E.err || { tail -20 $OUT/E.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/E.$i.json'));print('E', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o E -- python3 bench.py --config E --steps 12 --warmup 2 --no-cpu-baseline > $OUT/prof.log 2>&1 || exit 1
find $OUT/prof -name "*kernel_stats.csv" | head -1
