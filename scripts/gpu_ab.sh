#!/bin/bash
# Scratch A/B of two library builds (rewritten per experiment): the default
# in-tree library against $OLD (CG_LIB_PATH), bench lines interleaved.
#   bash scripts/gpu_ab.sh TAG OLD.so
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-ab}
OLD=$GRAFT_REPO_ROOT/${2:-cnn_graph_amd/libcheb_old.so}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused_adam.py -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1; echo "pytest rc=$?"
tail -1 $OUT/pytest.txt
for i in 1 2 3; do
timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > $OUT/new.$i.json 2>$OUT/b.err || { echo BENCH_FAIL; tail -20 $OUT/b.err; exit 1; }
CG_LIB_PATH=$OLD timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline > $OUT/old.$i.json 2>$OUT/b.err || { echo BENCH_FAIL; tail -20 $OUT/b.err; exit 1; }
for v in new old; do python3 -c "import json;d=json.load(open('$OUT/$v.$i.json'));print('$v', d['value'], d['ms_per_step'], d['kernels']['fwd']['avg_ms'], d['kernels']['bwd']['avg_ms'])"; done
done
