#!/bin/bash
# GPU pass: smoke, parity tests, bench, optional rocprofv3 kernel trace.
#   bash scripts/gpu_check.sh [tag] [prof]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 8 > $OUT/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
if [ "$2" == "prof" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o kt --output-format csv -- python3 bench.py --steps 100 --warmup 10 --no-cpu-baseline > $OUT/prof.log 2>&1 || { echo PROF_FAIL; tail -30 $OUT/prof.log; exit 1; }
  find $OUT/prof -name "*kernel_stats.csv" -exec cat {} \; | head -20
fi
