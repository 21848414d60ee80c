#!/bin/bash
# r04: k_lstm_seq2 with x staged in LDS, c_{t-1} with the tile loads and
# pipelined weight reads: LSTM tests, E A/B (CG_SEQ_V=2/1), seq2 stamps.
#   bash scripts/gpu_r04_k.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_k}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_lstm.py > $O/pytest.txt 2>&1
rc=$?; tail -5 $O/pytest.txt; [ $rc -le 1 ] || exit 1
for rep in 1 2; do
  for v in 2 1; do
    CG_SEQ_V=$v timeout -k 10 200 python3 scripts/bench_configs.py E --no-cpu >> $O/E_seq$v.jsonl 2>> $O/E.err || { tail -5 $O/E.err; exit 1; }
  done
done
for v in 2 1; do echo "== CG_SEQ_V=$v"; cut -c1-200 $O/E_seq$v.jsonl; done
for f in 0 1 192; do
  CG_SEQ_V=2 timeout -k 10 120 python3 scripts/stamps_E.py $f >> $O/stampsE.jsonl 2>> $O/E.err || { tail -5 $O/E.err; exit 1; }
done
cat $O/stampsE.jsonl
echo DONE
