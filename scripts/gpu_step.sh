#!/bin/bash
# Scratch GPU pass for the current iteration (rewritten per call; see DESIGN.md
# for the measured numbers it produced).   bash scripts/gpu_step.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-step}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused_adam.py -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1; echo "pytest rc=$?"
tail -3 $OUT/pytest.txt | cut -c1-300
grep -E "^(FAILED|ERROR)|^E  " $OUT/pytest.txt | head -20 | cut -c1-300
for i in 1 2 3; do
for v in 0 1; do
timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --opt gemm_x3=$v > $OUT/b$v.$i.json 2>$OUT/b.err || { echo BENCH_FAIL; tail -20 $OUT/b.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/b$v.$i.json'));print('x3=$v', d['value'], d['ms_per_step'], d['kernels']['fwd']['avg_ms'], d['kernels']['bwd']['avg_ms'])"
done
done
