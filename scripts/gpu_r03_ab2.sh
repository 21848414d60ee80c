#!/bin/bash
# r03: full -m gpu suite, then A/Bs: fused-dBasis Clenshaw (CG_CLEN_DY 0/1/2), k_dw_slabs rows per
# batch (CG_DW_RB 32/16), the MFMA/SpMM wave phases (CG_GRP_PHASE, CG_SEQ_PHASE 1/0)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_ab2}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
tail -2 $O/pytest.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest.txt | head; exit 1; }
for rep in 1 2; do
  for v in 0 1 2; do
    CG_CLEN_DY=$v timeout -k 10 120 python3 scripts/clen_ab.py >> $O/clen_ab.txt 2>&1 || exit 1
  done
done
grep backward $O/clen_ab.txt
for rep in 1 2; do
  for v in base rb16 grp0 seq0; do
    case $v in
      base) E="" ;; rb16) E="CG_DW_RB=16" ;; grp0) E="CG_GRP_PHASE=0" ;; seq0) E="CG_SEQ_PHASE=0" ;;
    esac
    env $E timeout -k 10 300 python3 scripts/bench_configs.py R E C2 >> $O/cfg_$v.jsonl 2>> $O/cfg.err || exit 1
  done
done
for v in base rb16 grp0 seq0; do echo "== $v"; cut -c1-200 $O/cfg_$v.jsonl; done
