#!/bin/bash
# r04: config R's group kernels -- phase stamps (debug build) of k_grp16_fwd / k_grp_clen_dy,
# packed-column k_grp_clen A/B (CG_CLEN_DY=0, CG_GRP_PC=1/0), then the LDS attribution of
# cheb_fwd_fast (scripts/gpu_r04_lds.sh).   bash scripts/gpu_r04_grp.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_grp}
mkdir -p $O
timeout -k 10 200 python3 scripts/stamps_R.py > $O/stampsR.json 2> $O/stampsR.err || { tail -5 $O/stampsR.err; exit 1; }
cat $O/stampsR.json
for rep in 1 2; do
  for v in 1 0; do
    CG_CLEN_DY=0 CG_GRP_PC=$v timeout -k 10 120 python3 scripts/clen_ab.py >> $O/clen_pc$v.txt 2>> $O/clen.err || { tail -5 $O/clen.err; exit 1; }
  done
done
for v in 1 0; do echo "== CG_GRP_PC=$v"; cat $O/clen_pc$v.txt; done
bash scripts/gpu_r04_lds.sh ${1:-r04_grp}/lds > $O/lds.log 2>&1 || { tail -20 $O/lds.log; exit 1; }
tail -40 $O/lds.log
echo DONE
