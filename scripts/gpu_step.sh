#!/bin/bash
# Scratch GPU pass for the current iteration (rewritten per call; see DESIGN.md
# for the measured numbers it produced).   bash scripts/gpu_step.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-step}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest.txt | cut -c1-400; exit 1; }
tail -1 $OUT/pytest.txt
for i in 1 2; do
timeout -k 10 300 python scripts/bench_configs.py E --no-cpu --opt dw_x3=0 > $OUT/E_f32.$i.jsonl 2>$OUT/cfg.err || { echo CFG_FAIL; tail -20 $OUT/cfg.err; exit 1; }
timeout -k 10 300 python scripts/bench_configs.py E --no-cpu > $OUT/E_x3.$i.jsonl 2>$OUT/cfg.err || { echo CFG_FAIL; tail -20 $OUT/cfg.err; exit 1; }
done
cut -c1-200 $OUT/E_*.jsonl
timeout -k 10 300 python bench.py --config E --steps 30 --warmup 3 --no-cpu-baseline > $OUT/bench_E.json 2>$OUT/bE.err || { echo BE_FAIL; tail -20 $OUT/bE.err; exit 1; }
cut -c1-300 $OUT/bench_E.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ktE -o E --output-format csv -- python3 scripts/bench_configs.py E --no-cpu > $OUT/ktE.log 2>&1 || { echo KTE_FAIL; tail -20 $OUT/ktE.log; exit 1; }
python3 -c "
import csv
for r in list(csv.DictReader(open('$OUT/ktE/E_kernel_stats.csv')))[:6]: print(r['Name'][:60], r['Calls'], r['AverageNs'])"
