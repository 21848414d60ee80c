#!/bin/bash
# gconv-LSTM x basis precomputed for all steps: bitwise A/B, LSTM tests, E timing A/B, bench stdout
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_xpre}
mkdir -p $O
timeout -k 10 300 python3 scripts/seq_xpre_check.py > $O/xpre_check.txt 2>&1 || { tail -20 $O/xpre_check.txt; exit 1; }
grep -v amdgpu.ids $O/xpre_check.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_lstm.py -x -q --tb=short --timeout 200 --timeout-method thread > $O/pytest_lstm.txt 2>&1 || { tail -30 $O/pytest_lstm.txt; exit 1; }
tail -1 $O/pytest_lstm.txt
for rep in 1 2; do
  for v in 1 0; do
    CG_SEQ_XPRE=$v timeout -k 10 200 python3 scripts/bench_configs.py E >> $O/E_xpre$v.jsonl 2>> $O/E.err || exit 1
  done
done
for v in 1 0; do echo "== xpre $v"; cut -c1-200 $O/E_xpre$v.jsonl; done
timeout -k 10 200 python3 bench.py --force-allreduce --no-cpu-baseline > $O/bench_ar.json 2> $O/bench_ar.err || exit 1
echo "stdout lines: $(wc -l < $O/bench_ar.json)"; head -c 150 $O/bench_ar.json; echo
