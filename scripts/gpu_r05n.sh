#!/bin/bash
# group / model / epilogue tests, config R timing + kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05n}
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_group.py tests/test_gpu_model.py tests/test_gpu_dense.py tests/test_gpu_basis_layout.py > $OUT/pytest.txt 2>&1 || { echo TEST_FAIL; tail -60 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
timeout -k 10 300 python scripts/bench_configs.py R R --no-cpu > $OUT/R.jsonl 2>&1 || { echo R_FAIL; tail -20 $OUT/R.jsonl; exit 1; }
cat $OUT/R.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o R --output-format csv -- python3 scripts/bench_configs.py R --no-cpu > $OUT/kt.log 2>&1 || { echo KT_FAIL; tail -20 $OUT/kt.log; exit 1; }
find $OUT/kt -name "*kernel_stats.csv" -exec head -10 {} \;
