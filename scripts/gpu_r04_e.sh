#!/bin/bash
# r04: (1) GPU tests touched this round (dW direct, LSTM, fast path layout), (2)
# config E phase ablation of k_lstm_seq / k_lstm_seq2 (debug build stamps),
# (3) cheb_fwd_fast LDS bank conflicts on the conflict-free layout + the bench.
#   bash scripts/gpu_r04_e.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_e}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
  tests > $O/pytest.txt 2>&1
rc=$?; tail -5 $O/pytest.txt; [ $rc -le 1 ] || exit 1
for v in 1 2; do
  for f in 0 1 4 16 448 469 2; do
    CG_SEQ_V=$v timeout -k 10 120 python3 scripts/stamps_E.py $f >> $O/stampsE.jsonl 2>> $O/E.err || { tail -5 $O/E.err; exit 1; }
  done
done
cat $O/stampsE.jsonl
bash scripts/gpu_r04_lds.sh ${1:-r04_e}/lds > $O/lds.log 2>&1 || { tail -20 $O/lds.log; exit 1; }
tail -42 $O/lds.log
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cut -c1-400 $O/bench.json
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['kernels'], d['roofline']['frac'], d['roofline_spmm_fwd']['frac'])"
echo DONE
