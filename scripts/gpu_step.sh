#!/bin/bash
# Scratch GPU pass for the current iteration (rewritten per call; see DESIGN.md
# for the measured numbers it produced).   bash scripts/gpu_step.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-step}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused_adam.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest.txt | cut -c1-300; exit 1; }
tail -1 $OUT/pytest.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/ktA -o A --output-format csv -- python3 scripts/bench_configs.py A --no-cpu > $OUT/ktA.log 2>&1 || { echo KTA_FAIL; tail -20 $OUT/ktA.log; exit 1; }
grep config $OUT/ktA.log
python3 -c "
import csv
for r in list(csv.DictReader(open('$OUT/ktA/A_kernel_stats.csv')))[:4]: print(r['Name'][:60], r['AverageNs'])"
