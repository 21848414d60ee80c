#!/bin/bash
# End-of-round GPU pass, part 2: every configuration's timing with its CPU leg, C2 / D in the
# planes layout, a kernel trace of config R, and the bench's kernel trace + PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python scripts/bench_configs.py A C1 C2 D E R > $OUT/configs.jsonl 2>&1 || { echo CFG_FAIL; tail -20 $OUT/configs.jsonl; exit 1; }
grep config $OUT/configs.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ktR -o R --output-format csv -- python3 scripts/bench_configs.py R --no-cpu > $OUT/ktR.log 2>&1 || { echo KTR_FAIL; tail -20 $OUT/ktR.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ktE -o E --output-format csv -- python3 scripts/bench_configs.py E --no-cpu > $OUT/ktE.log 2>&1 || { echo KTE_FAIL; tail -20 $OUT/ktE.log; exit 1; }
bash scripts/prof_pmc.sh $TAG/pmc > $OUT/pmc.log 2>&1 || { echo PMC_FAIL; tail -20 $OUT/pmc.log; exit 1; }
tail -5 $OUT/pmc.log
