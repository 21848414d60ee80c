#!/bin/bash
# Scratch GPU pass for the current iteration (rewritten per call; see DESIGN.md
# for the measured numbers it produced).   bash scripts/gpu_step.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-step}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_adam.py tests/test_gpu_slab_reduce.py tests/test_gpu_dp_bench.py -k "not config_de and not config_e" -x -v --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest.txt | cut -c1-300; exit 1; }
tail -1 $OUT/pytest.txt
for i in 1 2 3; do
for sc in fused deferred; do
timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --schedule $sc > $OUT/bench_$sc.$i.json 2>$OUT/bench.err || { echo BENCH_FAIL; tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_$sc.$i.json'));print('$sc', d['value'], d['ms_per_step'], d['kernels']['fwd']['avg_ms'], d['kernels']['bwd']['avg_ms'])"
done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/ktB -o B --output-format csv -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline > $OUT/ktB.log 2>&1 || { echo KTB_FAIL; tail -20 $OUT/ktB.log; exit 1; }
python3 -c "
import csv
for r in list(csv.DictReader(open('$OUT/ktB/B_kernel_stats.csv')))[:4]: print(r['Name'][:60], r['Calls'], r['AverageNs'])"
