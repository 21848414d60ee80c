#!/bin/bash
# r04: config R side-stream dW A/B (CG_SIDE_DW=0/1) + its bitwise test, R phase
# stamps, config E phase ablation of k_lstm_seq / k_lstm_seq2 (flags in the
# sequence kernels' debug byte).   bash scripts/gpu_r04_f.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_f}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_group.py tests/test_gpu_model.py > $O/pytest.txt 2>&1
rc=$?; tail -5 $O/pytest.txt; [ $rc -le 1 ] || exit 1
for rep in 1 2; do
  for v in 1 0; do
    CG_SIDE_DW=$v timeout -k 10 200 python3 scripts/bench_configs.py R --no-cpu >> $O/R_side$v.jsonl 2>> $O/R.err || { tail -5 $O/R.err; exit 1; }
  done
done
for v in 1 0; do echo "== CG_SIDE_DW=$v"; cut -c1-250 $O/R_side$v.jsonl; done
timeout -k 10 200 python3 scripts/stamps_R.py > $O/stampsR.json 2> $O/stampsR.err || { tail -5 $O/stampsR.err; exit 1; }
cat $O/stampsR.json
for v in 1 2; do
  for f in 0 1 2 4 16 192 213; do
    CG_SEQ_V=$v timeout -k 10 120 python3 scripts/stamps_E.py $f >> $O/stampsE.jsonl 2>> $O/E.err || { tail -5 $O/E.err; exit 1; }
  done
done
cat $O/stampsE.jsonl
echo DONE
