#!/bin/bash
# r03: LSTM tests + seq ablations + config E timing
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-r03_lstm2}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_lstm.py -x -v --tb=short --timeout 200 --timeout-method thread > $O/pytest_lstm.txt 2>&1; rc=$?
grep -E "FAIL|Error|passed|failed" $O/pytest_lstm.txt | tail -20
[ $rc -eq 0 ] || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 300 python3 scripts/ablate_lstm.py > $O/ablate_lstm.json 2> $O/ablate_lstm.err && cat $O/ablate_lstm.json &&
timeout -k 10 300 python3 scripts/bench_configs.py E E_step > $O/configE.jsonl 2> $O/configE.err && cat $O/configE.jsonl
