#!/bin/bash
# config E phase stamps on the debug build (ablation flags), then config D PMC passes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05d}
mkdir -p $OUT
for F in 0 1 2 4 16 192 213; do
  CG_LIB_PATH=scripts/ablib/dbg.so timeout -k 10 120 python scripts/stamps_E.py $F >> $OUT/stampsE.jsonl 2> $OUT/stampsE_$F.err || { echo STAMP_FAIL $F; tail -20 $OUT/stampsE_$F.err; exit 1; }
done
cat $OUT/stampsE.jsonl
bash scripts/gpu_r05_dpmc.sh r05_dpmc
