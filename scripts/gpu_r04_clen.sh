#!/bin/bash
# r04: config R's k_grp_clen_dy ablation (debug build stamps; flags 1 no D-tile
# MFMAs, 2 no SpMM, 4 no dy loads, 8 no hand-over).   bash scripts/gpu_r04_clen.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_clen}
mkdir -p $O
for f in 0 1 2 4 8 15; do
  timeout -k 10 200 python3 scripts/stamps_R.py $f bwd >> $O/stampsR.jsonl 2>> $O/R.err || { tail -5 $O/R.err; exit 1; }
done
cut -c1-400 $O/stampsR.jsonl
echo DONE
