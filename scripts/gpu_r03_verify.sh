#!/bin/bash
# r03 re-entry check of the committed tree: smoke, every -m gpu test, the default bench line,
# configs C1 C2 E R.   bash scripts/gpu_r03_verify.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-r03_verify}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --tb=short --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
grep -E "FAIL|Error|passed|failed" $O/pytest.txt | tail -20
[ $rc -eq 0 ] || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err && cat $O/bench.json &&
timeout -k 10 400 python3 scripts/bench_configs.py C1 C2 E R > $O/configs.jsonl 2> $O/configs.err && cat $O/configs.jsonl
