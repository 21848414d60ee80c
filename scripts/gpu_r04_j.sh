#!/bin/bash
# r04: k_dw_direct two-waves-per-SIMD build (CG_DW_W2=1/0): bitwise tests, then
# A/B on configs C2 and E (the wgrad pass) with kernel traces.   bash scripts/gpu_r04_j.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_j}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_dw_direct.py > $O/pytest.txt 2>&1
rc=$?; tail -5 $O/pytest.txt; [ $rc -le 1 ] || exit 1
for v in 1 0; do
  CG_DW_W2=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt$v -o kt --output-format csv -- python3 scripts/bench_configs.py C2 E --no-cpu > $O/ab$v.jsonl 2> $O/ab$v.err || { tail -20 $O/ab$v.err; exit 1; }
  python3 - <<PY
import csv, glob
rows = [r for p in glob.glob("$O/kt$v/**/*kernel_stats.csv", recursive=True) for r in csv.DictReader(open(p))]
print("== CG_DW_W2=$v")
for r in rows:
    if "dw_direct" in r["Name"] or "dw_slabs" in r["Name"]:
        print(f'{r["Name"][:80]:80s} calls {r["Calls"]:>5s} avg_us {float(r["AverageNs"])/1e3:9.1f}')
PY
  grep '^{' $O/ab$v.jsonl | cut -c1-200
done
echo DONE
