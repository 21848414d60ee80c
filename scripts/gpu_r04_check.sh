#!/bin/bash
# r04 check pass: smoke, every -m gpu test (captured output of passing tests
# shown: the config-R per-filter test prints its ReLU-mask flip counts), the
# default bench line.   bash scripts/gpu_r04_check.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_check}
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 1100 python -u -m pytest tests -m gpu -v -rP --tb=short --timeout 240 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
grep -E "passed|failed" $O/pytest.txt | tail -2
# a failing assertion is reported and the pass goes on; a hang / crash (timeout, signal) ends it
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/pytest.txt | head -30; [ $rc -eq 1 ] || exit 1; }
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
echo DONE
