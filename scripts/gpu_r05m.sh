#!/bin/bash
# BPTT-step ablation stamps (debug build)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05m}
mkdir -p $OUT
CG_LIB_PATH=scripts/ablib/dbg.so timeout -k 10 200 python scripts/ablate_bstep.py > $OUT/ablate_bstep.json 2> $OUT/ablate_bstep.err || { echo ABL_FAIL; tail -20 $OUT/ablate_bstep.err; exit 1; }
python3 -c "
import json
for k,v in json.load(open('$OUT/ablate_bstep.json')).items(): print(k, v)
"
