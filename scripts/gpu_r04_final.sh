#!/bin/bash
# r04 closing measurement on the committed tree: the default bench line, the driver's
# 20/5 command twice, the exchange schedule (--force-allreduce), then rocprofv3 kernel
# trace + PMC passes of the bench (scripts/prof_pmc.sh -> summary for profiles/pmc_latest.json)
#   bash scripts/gpu_r04_final.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-r04_final}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
for r in 1 2; do timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20_$r.json 2>> $O/bench.err || exit 1; done
timeout -k 10 200 python3 bench.py --force-allreduce --no-cpu-baseline > $O/bench_ar.json 2>> $O/bench.err || exit 1
python3 -c "
import json
for f in ['bench.json', 'bench20_1.json', 'bench20_2.json', 'bench_ar.json']:
    d = [json.loads(l) for l in open('$O/' + f) if l.startswith('{')][0]
    print(f, d['value'], d['ms_per_step'], d['step_ms_median'], d['roofline']['frac'], d['roofline_spmm_fwd']['frac'], d.get('cpu_baseline', {}).get('value'))"
bash scripts/prof_pmc.sh $TAG/pmc > $O/prof_pmc.log 2>&1 || { tail -20 $O/prof_pmc.log; exit 1; }
tail -30 $O/prof_pmc.log
echo DONE
