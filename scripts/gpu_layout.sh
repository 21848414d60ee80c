#!/bin/bash
# Orders basis layout on MI355X: its GPU tests + the fast-path parity tests,
# the bench with each layout on the same box, and a kernel trace of the
# orders-layout bench.   bash scripts/gpu_layout.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-layout}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_basis_layout.py tests/test_gpu_fused_adam.py tests/test_gpu_parity.py > $OUT/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for L in rows orders rows orders; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --basis-layout $L >> $OUT/bench_$L.json 2>$OUT/bench_$L.err || { echo BENCH_FAIL; tail -20 $OUT/bench_$L.err; exit 1; }
done
python3 - $OUT <<'PY'
import json, sys
for L in ("rows", "orders"):
    for line in open(f"{sys.argv[1]}/bench_{L}.json"):
        d = json.loads(line)
        k = d["kernels"]
        print(L, d["value"], d["ms_per_step"], "fwd", k["fwd"]["avg_ms"], "bwd", k["bwd"]["avg_ms"], "frac_fwd", d["roofline_spmm_fwd"]["frac"])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline > $OUT/kt.log 2>&1 || { echo KT_FAIL; tail -20 $OUT/kt.log; exit 1; }
find $OUT/kt -name "*kernel_stats.csv" | head -1 | xargs -I{} python3 -c "
import csv,sys
for r in csv.DictReader(open('{}')):
    print(r['Name'][:50], r['Calls'], r['AverageNs'])
" | head -6
