#!/bin/bash
# Bench-path GPU tests, two bench lines and a rocprofv3 kernel trace of the
# bench (per-kernel averages printed).   bash scripts/gpu_kt.sh TAG [bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-kt}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused_adam.py tests/test_gpu_parity.py tests/test_gpu_model.py > $OUT/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline "$@" >> $OUT/bench.json 2>$OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
done
cut -c1-160 $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline "$@" > $OUT/kt.log 2>&1 || { echo KT_FAIL; tail -20 $OUT/kt.log; exit 1; }
python3 - $OUT <<'PY'
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/kt/**/kt_kernel_stats.csv", recursive=True)[0]
for i, r in enumerate(csv.DictReader(open(f))):
    if i < 5:
        print(r["Name"][:60], r["Calls"], r["AverageNs"])
PY
