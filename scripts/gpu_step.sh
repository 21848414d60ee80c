#!/bin/bash
# Scratch GPU pass for the current iteration (rewritten per call; see DESIGN.md
# for the measured numbers it produced).   bash scripts/gpu_step.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-step}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo SMOKE_FAIL; tail -30 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.txt | cut -c1-300; exit 1; }
tail -1 $OUT/pytest_gpu.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/ktA -o A --output-format csv -- python3 scripts/bench_configs.py A --no-cpu > $OUT/ktA.log 2>&1 || { echo KTA_FAIL; tail -20 $OUT/ktA.log; exit 1; }
grep config $OUT/ktA.log
cut -d, -f1-4 $OUT/ktA/A_kernel_stats.csv | head -4 | cut -c1-150
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 10 > $OUT/bench.json 2>$OUT/bench.err || { echo BENCH_FAIL; tail -30 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-400
