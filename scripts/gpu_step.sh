#!/bin/bash
# Scratch GPU pass for the current iteration (rewritten per call; see DESIGN.md
# for the measured numbers it produced).   bash scripts/gpu_step.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-step}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1; echo "pytest rc=$?"
tail -15 $OUT/pytest.txt | cut -c1-300
grep -E "^(FAILED|ERROR)" $OUT/pytest.txt | head -20
timeout -k 10 400 python bench.py --config D --steps 4 --warmup 1 --no-cpu-baseline > $OUT/bD_x3.json 2>$OUT/bD.err || { echo BD_FAIL; tail -20 $OUT/bD.err; exit 1; }
timeout -k 10 400 python bench.py --config D --steps 4 --warmup 1 --no-cpu-baseline --opt gemm_x3=0 > $OUT/bD_f32.json 2>$OUT/bD.err || { echo BD_FAIL; tail -20 $OUT/bD.err; exit 1; }
cut -c1-260 $OUT/bD_x3.json $OUT/bD_f32.json
