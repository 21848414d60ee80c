#!/bin/bash
# r03 closing pass on the committed tree: smoke, every -m gpu test, the default bench line, the
# driver's 20/5 command, the exchange path (--force-allreduce: one-rank RCCL, rccl_nranks) and
# the HIP-graph replay option.   bash scripts/gpu_r03_close.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_close}
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
tail -1 $O/pytest.txt
[ $rc -eq 0 ] || { grep -E "FAIL|Error" $O/pytest.txt | head; exit 1; }
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2>> $O/bench.err || exit 1
for r in 2 3; do timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/bench_$r.json 2>> $O/bench.err || exit 1; done
timeout -k 10 200 python3 bench.py --force-allreduce --no-cpu-baseline > $O/bench_ar.json 2>> $O/bench.err || exit 1
timeout -k 10 200 python3 bench.py --graph on --no-cpu-baseline > $O/bench_graph.json 2>> $O/bench.err || exit 1
python3 -c "
import json
for f in ['bench.json', 'bench_2.json', 'bench_3.json', 'bench20.json', 'bench_ar.json', 'bench_graph.json']:
    d = [json.loads(l) for l in open('$O/' + f) if l.startswith('{')][0]; c = d['config']
    print(f, d['value'], d['ms_per_step'], d['step_ms_median'], d['roofline']['frac'], d['roofline_spmm_fwd']['frac'], c['allreduce'], c['rccl_nranks'], c['adam'][:30], c['launch'])"
timeout -k 10 400 python3 scripts/bench_configs.py C1 C2 E R > $O/configs.jsonl 2> $O/configs.err && cut -c1-220 $O/configs.jsonl
