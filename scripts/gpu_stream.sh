#!/bin/bash
# streaming-path pass: parity tests touching it, then config C/D/E timings
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-stream}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_lstm.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu > $OUT/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "Error|assert|FAIL" $OUT/pytest.log | head -30; tail -5 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 400 python scripts/bench_configs.py > $OUT/cfg.log 2>&1 || { tail -20 $OUT/cfg.log; exit 1; }
grep config $OUT/cfg.log
if [ "$2" == "prof" ]; then
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o kt --output-format csv -- python3 scripts/bench_configs.py C1 C2 D > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" -exec cut -c1-160 {} \; | head -12
fi
