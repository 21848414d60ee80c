#!/bin/bash
# r04: config D (planes, N = 256) backward kernel trace with k_dw_direct on (1), off (0) and
# with two-float basis loads (2: one column group, dy read once): per-kernel durations.   bash scripts/gpu_r04_d.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_d}
mkdir -p $O
for v in 1 0 2; do
  CG_DW_DIRECT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt$v -o kt --output-format csv -- python3 scripts/bench_configs.py D --d-batch 256 --layout planes --no-cpu > $O/D$v.log 2>&1 || { tail -20 $O/D$v.log; exit 1; }
  python3 - <<PY
import csv, glob
rows = [r for p in glob.glob("$O/kt$v/**/*kernel_stats.csv", recursive=True) for r in csv.DictReader(open(p))]
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
print("== CG_DW_DIRECT=$v")
for r in rows[:12]:
    print(f'{r["Name"][:70]:70s} calls {r["Calls"]:>5s} avg_ms {float(r["AverageNs"])/1e6:9.3f} total_ms {float(r["TotalDurationNs"])/1e6:9.2f}')
PY
done
echo DONE
