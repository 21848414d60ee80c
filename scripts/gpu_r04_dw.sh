#!/bin/bash
# r04: k_dw_direct vs k_dw_slabs (CG_DW_DIRECT=1/0) on configs C2, E, R and D at its
# per-rank batch (planes), then every config once with its CPU baseline leg.
#   bash scripts/gpu_r04_dw.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_dw}
mkdir -p $O
for rep in 1 2; do
  for v in 1 0; do
    CG_DW_DIRECT=$v timeout -k 10 300 python3 scripts/bench_configs.py C2 E R --no-cpu >> $O/ab_dw$v.jsonl 2>> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
  done
done
for v in 1 0; do
  CG_DW_DIRECT=$v timeout -k 10 300 python3 scripts/bench_configs.py D --d-batch 256 --layout planes --no-cpu >> $O/ab_dw$v.jsonl 2>> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
done
for v in 1 0; do echo "== CG_DW_DIRECT=$v"; cut -c1-230 $O/ab_dw$v.jsonl; done
timeout -k 10 600 python3 scripts/bench_configs.py C1 C2 E R > $O/configs.jsonl 2> $O/configs.err || { tail -5 $O/configs.err; exit 1; }
timeout -k 10 300 python3 scripts/bench_configs.py D --d-batch 256 --layout planes >> $O/configs.jsonl 2>> $O/configs.err || { tail -5 $O/configs.err; exit 1; }
python3 -c "
import json
for l in open('$O/configs.jsonl'):
    d = json.loads(l); c = d.get('cpu_baseline', {})
    print(d['config'], d.get('fwd_ms'), d.get('bwd_ms', d.get('fwd_bwd_ms', d.get('step_ms'))), d['samples_per_s'], 'cpu', c.get('value'), c.get('pass_ms_median'))"
timeout -k 10 300 python3 scripts/ablate_bstep.py > $O/ablate_bstep.json 2> $O/ablate_bstep.err || { tail -5 $O/ablate_bstep.err; exit 1; }
python3 -c "import json; d = json.load(open('$O/ablate_bstep.json')); [print(k, v) for k, v in d.items()]"
echo DONE
