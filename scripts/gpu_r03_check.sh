#!/bin/bash
# r03 checkpoint: the whole -m gpu suite, then configs E and R
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-r03_check}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --tb=short --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
grep -E "FAIL|Error|passed|failed" $O/pytest.txt | tail -20
[ $rc -eq 0 ] || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 300 python3 scripts/bench_configs.py E R > $O/configs.jsonl 2> $O/configs.err && cat $O/configs.jsonl
