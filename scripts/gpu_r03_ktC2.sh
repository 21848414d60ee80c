#!/bin/bash
# kernel traces of config C2 (rows and planes layouts)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_ktC2}
mkdir -p $O
for L in rows planes; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$L -o kt --output-format csv -- python3 scripts/bench_configs.py C2 --layout $L --rounds 1 > $O/kt_$L.log 2>&1 || { tail -20 $O/kt_$L.log; exit 1; }
  python3 scripts/pmc_table.py $O/kt_$L > $O/table_$L.json
  python3 -c "
import json; d=json.load(open('$O/table_$L.json'))['kernels']
for k,v in sorted(d.items(), key=lambda kv:-kv[1]['avg_us']*kv[1]['calls'])[:8]: print('$L', k, v['calls'], v['avg_us'])"
done
