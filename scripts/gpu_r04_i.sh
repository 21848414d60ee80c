#!/bin/bash
# r04: k_lstm_bstep with phase-A act loads one tile ahead: LSTM tests,
# E bench x2, bstep ablation.   bash scripts/gpu_r04_i.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_i}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_lstm.py > $O/pytest.txt 2>&1
rc=$?; tail -5 $O/pytest.txt; [ $rc -le 1 ] || exit 1
for rep in 1 2; do
  timeout -k 10 200 python3 scripts/bench_configs.py E --no-cpu >> $O/E.jsonl 2>> $O/E.err || { tail -5 $O/E.err; exit 1; }
done
cut -c1-220 $O/E.jsonl
timeout -k 10 300 python3 scripts/ablate_bstep.py > $O/ablate_bstep.json 2> $O/ablate_bstep.err || { tail -5 $O/ablate_bstep.err; exit 1; }
cat $O/ablate_bstep.json
echo DONE
