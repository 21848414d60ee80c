#!/bin/bash
# kernel-trace A/B of the fused-dBasis Clenshaw variants on config R's hidden-layer backward
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_clenab}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_group.py -x -q --timeout 120 --timeout-method thread > $O/pytest_group.txt 2>&1 || { tail -30 $O/pytest_group.txt; exit 1; }
tail -1 $O/pytest_group.txt
for rep in 1 2; do
  for v in 0 1 2; do
    CG_CLEN_DY=$v timeout -k 10 120 python3 scripts/clen_ab.py >> $O/ab.txt 2>&1 || exit 1
  done
done
cat $O/ab.txt | grep backward
for v in 0 1 2; do
  CG_CLEN_DY=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt$v -o kt --output-format csv -- python3 scripts/clen_ab.py > $O/kt$v.log 2>&1 || { tail $O/kt$v.log; exit 1; }
  python3 scripts/pmc_table.py $O/kt$v > $O/table$v.json
  python3 -c "
import json; d=json.load(open('$O/table$v.json'))['kernels']
print('$v', {k: (v['calls'], v['avg_us']) for k, v in d.items() if v['calls'] >= 30})"
done
# k_dw_slabs rows per batch: 32 (default) vs 16, configs R, E, C2 alternating
for rep in 1 2; do
  for v in 32 16; do
    CG_DW_RB=$v timeout -k 10 300 python3 scripts/bench_configs.py R E C2 >> $O/rb$v.jsonl 2>> $O/rb.err || exit 1
  done
done
for v in 32 16; do echo "== RB $v"; cut -c1-260 $O/rb$v.jsonl; done
