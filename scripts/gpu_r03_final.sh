#!/bin/bash
# r03 final pass on the committed tree: smoke, every -m gpu test, the default bench line and the
# driver's 20/5 command, rocprofv3 kernel trace + PMC passes of the bench, configs C1 C2 E R and
# D at its per-rank batch, a kernel trace + PMC passes of config R.   bash scripts/gpu_r03_final.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-r03_final}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
tail -1 $O/pytest.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest.txt | head; exit 1; }
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
for r in 1 2; do timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20_$r.json 2>> $O/bench.err || exit 1; done
python3 -c "
import json
for f in ['bench.json', 'bench20_1.json', 'bench20_2.json']:
    d = json.load(open('$O/' + f)); print(f, d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_spmm_fwd']['frac'], d.get('cpu_baseline', {}).get('value'))"
bash scripts/prof_pmc.sh $TAG/pmc > $O/prof_pmc.log 2>&1 || { tail -20 $O/prof_pmc.log; exit 1; }
echo PMC_OK
timeout -k 10 400 python3 scripts/bench_configs.py C1 C2 E R > $O/configs.jsonl 2> $O/configs.err && cut -c1-220 $O/configs.jsonl || exit 1
timeout -k 10 400 python3 scripts/bench_configs.py D --d-batch 256 --layout planes > $O/D256.jsonl 2> $O/D256.err && cut -c1-260 $O/D256.jsonl || exit 1
bash scripts/gpu_r03_profER.sh $TAG/prof R > $O/profR.log 2>&1 || { tail -20 $O/profR.log; exit 1; }

# A/B: act stores staged through LDS (CG_SEQ_STAGE 1, default) vs per lane (0), config E
for rep in 1 2; do
  for v in 1 0; do
    CG_SEQ_STAGE=$v timeout -k 10 200 python3 scripts/bench_configs.py E >> $O/E_stage$v.jsonl 2>> $O/E_stage.err || exit 1
  done
done
for v in 1 0; do echo "== stage $v"; cut -c1-200 $O/E_stage$v.jsonl; done
echo DONE
