#!/bin/bash
# r04: config E's k_lstm_seq2 vs k_lstm_seq (CG_SEQ_V=2/1), config R's group kernels -- phase stamps (debug build) of k_grp16_fwd / k_grp_clen_dy,
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
for rep in 1 2; do
  for v in 2 1; do
    CG_SEQ_V=$v timeout -k 10 200 python3 scripts/bench_configs.py E --no-cpu >> $O/E_seq$v.jsonl 2>> $O/E.err || { tail -5 $O/E.err; exit 1; }
  done
done
for v in 2 1; do echo "== CG_SEQ_V=$v"; cut -c1-200 $O/E_seq$v.jsonl; done
for v in 2 1; do CG_SEQ_V=$v timeout -k 10 200 python3 scripts/stamps_E.py >> $O/stampsE.jsonl 2>> $O/E.err || { tail -5 $O/E.err; exit 1; }; done
cat $O/stampsE.jsonl
bash scripts/gpu_r04_lds.sh ${1:-r04_grp}/lds > $O/lds.log 2>&1 || { tail -20 $O/lds.log; exit 1; }
tail -40 $O/lds.log
echo DONE
