#!/bin/bash
# quick GPU pass: parity tests + ablation + bench (no rocprof)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-quick}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -x -q > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 200 python scripts/ablate.py > $OUT/ablate.json 2>&1 || { echo ABLATE_FAIL; tail -20 $OUT/ablate.json; exit 1; }
cat $OUT/ablate.json | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
