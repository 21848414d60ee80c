#!/bin/bash
# r03: full -m gpu suite, then the double-buffered k_dw_slabs A/B (CG_DW_DB 1/0) on R E C2 D
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_db}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
tail -2 $O/pytest.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest.txt | head; exit 1; }
for rep in 1 2; do
  for v in 1 0; do
    CG_DW_DB=$v timeout -k 10 300 python3 scripts/bench_configs.py R E C2 D >> $O/db$v.jsonl 2>> $O/db.err || exit 1
  done
done
for v in 1 0; do echo "== DB $v"; cut -c1-230 $O/db$v.jsonl; done
