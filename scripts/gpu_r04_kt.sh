#!/bin/bash
# r04: per-kernel traces of configs E, R and C2 (rocprofv3 kernel trace + stats).
#   bash scripts/gpu_r04_kt.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_kt}
mkdir -p $O
for C in E R C2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt$C -o kt --output-format csv -- python3 scripts/bench_configs.py $C --no-cpu > $O/$C.log 2>&1 || { tail -20 $O/$C.log; exit 1; }
  python3 - <<PY
import csv, glob
rows = [r for p in glob.glob("$O/kt$C/**/*kernel_stats.csv", recursive=True) for r in csv.DictReader(open(p))]
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
print("== $C")
for r in rows[:14]:
    print(f'{r["Name"][:80]:80s} calls {r["Calls"]:>5s} avg_us {float(r["AverageNs"])/1e3:9.1f} total_ms {float(r["TotalDurationNs"])/1e6:9.2f}')
PY
done
echo DONE
