#!/bin/bash
# r04: config R's k_grp16_fwd ablation (debug build stamps, flags 0/1/2/4/7).
#   bash scripts/gpu_r04_r.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_r}
mkdir -p $O
for f in 0 1 2 4 7; do
  timeout -k 10 200 python3 scripts/stamps_R.py $f >> $O/stampsR.jsonl 2>> $O/R.err || { tail -5 $O/R.err; exit 1; }
done
cat $O/stampsR.jsonl
echo DONE
