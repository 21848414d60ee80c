#!/bin/bash
# r04: the whole -m gpu suite, smoke(), then every config's bench line with its
# CPU baseline leg -> configs.jsonl.   bash scripts/gpu_r04_configs.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_configs}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest.txt 2>&1
rc=$?; tail -5 $O/pytest.txt; [ $rc -le 1 ] || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
cat $O/smoke.txt | tail -2
timeout -k 10 900 python3 scripts/bench_configs.py A C1 C2 E R > $O/configs.jsonl 2> $O/configs.err || { tail -5 $O/configs.err; exit 1; }
timeout -k 10 400 python3 scripts/bench_configs.py D --d-batch 256 >> $O/configs.jsonl 2>> $O/configs.err || { tail -5 $O/configs.err; exit 1; }
python3 -c "
import json
for l in open('$O/configs.jsonl'):
    d = json.loads(l); c = d.get('cpu_baseline', {})
    print(d['config'], d.get('basis_layout', ''), d.get('fwd_ms'), d.get('bwd_ms', d.get('fwd_bwd_ms', d.get('step_ms'))), d['samples_per_s'], 'cpu', c.get('value'), c.get('unit'))"
echo DONE
