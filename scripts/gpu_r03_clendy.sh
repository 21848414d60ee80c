#!/bin/bash
# fused-dBasis Clenshaw (k_grp_clen_dy): new tests, bitwise A/B vs the row GEMM + k_grp_clen pair,
# the whole -m gpu suite, config R A/B (alternating), the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_clendy}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_group.py -x -v --tb=short --timeout 120 --timeout-method thread > $O/pytest_group.txt 2>&1; rc=$?
grep -E "PASS|FAIL|Error|passed|failed" $O/pytest_group.txt | tail -12
[ $rc -eq 0 ] || { tail -40 $O/pytest_group.txt; exit 1; }
timeout -k 10 300 python3 scripts/clen_dy_check.py > $O/clen_dy_check.txt 2>&1 || { tail -20 $O/clen_dy_check.txt; exit 1; }
cat $O/clen_dy_check.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q ${FULL_SUITE_SKIP:+--co} --tb=short --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
tail -3 $O/pytest.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest.txt | head; exit 1; }
for rep in 1 2; do
  for v in 1 0; do
    CG_CLEN_DY=$v timeout -k 10 200 python3 scripts/bench_configs.py R >> $O/R_clendy$v.jsonl 2>> $O/R.err || exit 1
  done
done
cat $O/R_clendy1.jsonl $O/R_clendy0.jsonl | cut -c1-300
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err && cat $O/bench.json | cut -c1-400
