#!/bin/bash
# A/B: bench timed region as eager C-ABI calls vs one HIP graph replay (driver's 20/5 and 200/20)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_graph}
mkdir -p $O
for rep in 1 2 3; do
  for g in off on; do
    timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --graph $g --no-cpu-baseline > $O/b20_${g}_$rep.json 2> $O/b20_${g}_$rep.err || { cat $O/b20_${g}_$rep.err | tail -20; exit 1; }
    timeout -k 10 120 python3 bench.py --steps 200 --warmup 20 --graph $g --no-cpu-baseline > $O/b200_${g}_$rep.json 2> $O/b200_${g}_$rep.err || exit 1
  done
done
for f in $O/b*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['config']['launch'])"; done
