#!/bin/bash
# fused-dBasis Clenshaw for Fout = 2 (the ResGNN output layer): group tests, bitwise A/B shapes,
# the whole -m gpu suite, config R A/B (CG_CLEN_DY 1/0)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_fout2}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_group.py -x -q --tb=short --timeout 120 --timeout-method thread > $O/pytest_group.txt 2>&1 || { tail -30 $O/pytest_group.txt; exit 1; }
tail -1 $O/pytest_group.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
tail -1 $O/pytest.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest.txt | head; exit 1; }
for rep in 1 2; do
  for v in 1 0; do
    CG_CLEN_DY=$v timeout -k 10 200 python3 scripts/bench_configs.py R >> $O/R_clendy$v.jsonl 2>> $O/R.err || exit 1
  done
done
for v in 1 0; do echo "== clen_dy $v"; cut -c1-200 $O/R_clendy$v.jsonl; done
