#!/bin/bash
# r04 closing check on the committed tree: the whole -m gpu suite, smoke(),
# the default bench line + the driver's 20/5 command, then config E's
# paired-row A/B (default library vs scripts/dbg/libcheb_alt_{b,c}.so).
#   bash scripts/gpu_r04_final2.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_final2}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest.txt 2>&1
rc=$?; tail -3 $O/pytest.txt; [ $rc -le 1 ] || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 300 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2>> $O/bench.err || exit 1
python3 -c "
import json
for f in ['bench.json', 'bench20.json']:
    d = [json.loads(l) for l in open('$O/' + f) if l.startswith('{')][0]
    print(f, d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_spmm_fwd']['frac'], d.get('cpu_baseline', {}).get('value'))"
for rep in 1 2; do
  for v in def alt_b alt_c; do
    if [ $v = def ]; then L=""; else L=$PWD/scripts/dbg/libcheb_$v.so; fi
    [ $v = def ] || [ -f "$L" ] || continue
    CG_LIB_PATH=$L timeout -k 10 200 python3 scripts/bench_configs.py E --no-cpu > $O/tmp.json 2>> $O/E.err || { tail -5 $O/E.err; exit 1; }
    echo "$v $(cut -c1-200 $O/tmp.json)" >> $O/E_ab.txt
  done
done
cat $O/E_ab.txt
echo DONE
