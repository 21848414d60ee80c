#!/bin/bash
# End-of-round GPU pass, part 1: smoke, every -m gpu test, the bench line (with the CPU baseline).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo SMOKE_FAIL; tail -30 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.txt; exit 1; }
tail -1 $OUT/pytest_gpu.txt
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 10 > $OUT/bench.json 2>&1 || { echo BENCH_FAIL; tail -30 $OUT/bench.json; exit 1; }
tail -1 $OUT/bench.json
