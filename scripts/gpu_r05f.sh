#!/bin/bash
# config E phase stamps on the debug build (ablation flags)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05f}
mkdir -p $OUT
shift
for F in "$@"; do
  CG_LIB_PATH=scripts/ablib/dbg.so timeout -k 10 120 python scripts/stamps_E.py $F >> $OUT/stampsE.jsonl 2> $OUT/stampsE_$F.err || { echo STAMP_FAIL $F; tail -20 $OUT/stampsE_$F.err; exit 1; }
done
cat $OUT/stampsE.jsonl
