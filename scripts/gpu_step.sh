#!/bin/bash
# Scratch GPU pass for the current iteration (rewritten per call; see DESIGN.md
# for the measured numbers it produced).   bash scripts/gpu_step.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-step}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_lstm.py tests/test_gpu_glstm_dp.py -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1; echo "pytest rc=$?"
tail -3 $OUT/pytest.txt | cut -c1-300
grep -E "^(FAILED|ERROR)|^E  " $OUT/pytest.txt | head -20 | cut -c1-300
for i in 1 2; do
timeout -k 10 300 python scripts/bench_configs.py E --no-cpu --opt gemm_x3=0 > $OUT/E_f32.$i.jsonl 2>$OUT/cfg.err || { echo CFG_FAIL; tail -20 $OUT/cfg.err; exit 1; }
timeout -k 10 300 python scripts/bench_configs.py E --no-cpu > $OUT/E_x3.$i.jsonl 2>$OUT/cfg.err || { echo CFG_FAIL; tail -20 $OUT/cfg.err; exit 1; }
done
cut -c1-200 $OUT/E_*.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ktE -o E --output-format csv -- python3 scripts/bench_configs.py E --no-cpu > $OUT/ktE.log 2>&1 || { echo KTE_FAIL; tail -20 $OUT/ktE.log; exit 1; }
python3 -c "
import csv
for r in list(csv.DictReader(open('$OUT/ktE/E_kernel_stats.csv')))[:6]: print(r['Name'][:60], r['Calls'], r['AverageNs'])"
