#!/bin/bash
# One GPU pass: smoke, every -m gpu test, kernel ablations, the bench line and a
# rocprofv3 kernel trace of the bench.  Stops at the first failing step.
#   bash scripts/gpu_round.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-round}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo SMOKE_FAIL; tail -30 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.txt; exit 1; }
tail -1 $OUT/pytest_gpu.txt
timeout -k 10 240 python scripts/ablate.py > $OUT/ablate.json 2>&1 || { echo ABLATE_FAIL; tail -20 $OUT/ablate.json; exit 1; }
grep -v amdgpu.ids $OUT/ablate.json | head -30
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 10 > $OUT/bench.json 2>&1 || { echo BENCH_FAIL; tail -30 $OUT/bench.json; exit 1; }
tail -1 $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline > $OUT/kt.txt 2>&1 || { echo PROF_FAIL; tail -30 $OUT/kt.txt; exit 1; }
find $OUT/kt -name "*kernel_stats.csv" -exec cut -c1-160 {} \; | head -12
