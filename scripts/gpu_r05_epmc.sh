#!/bin/bash
# Config E: PMC passes (FETCH_SIZE, WRITE_SIZE, TCC hit / miss, MFMA busy), each its own rocprofv3 run
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05_epmc}
mkdir -p $OUT
CMD="scripts/bench_configs.py E --no-cpu"
for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES"; do
  N=$(echo $C | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/pmc_$N -o pmc --output-format csv -- python3 $CMD > $OUT/pmc_$N.log 2>&1 || { echo "PMC_FAIL $C"; tail -20 $OUT/pmc_$N.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, re, json, sys
from collections import defaultdict
root = sys.argv[1]
out = defaultdict(lambda: defaultdict(list))
for f in glob.glob(root + '/**/*counter_collection.csv', recursive=True):
    for row in csv.DictReader(open(f)):
        k = re.search(r'(k_\w+|cheb_\w+|__amd\w+)', row.get('Kernel_Name', ''))
        k = k.group(1) if k else row.get('Kernel_Name', '')[:30]
        out[k][row['Counter_Name']].append(float(row['Counter_Value']))
res = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in out.items()}
json.dump(res, open(root + '/pmc_avg.json', 'w'), indent=1)
for k, d in res.items():
    print(k, {c: round(v, 1) for c, v in d.items()})
PY
