#!/bin/bash
# Scratch GPU step (rewritten per experiment): config E new library vs
# $OLD (CG_LIB_PATH), then the LSTM tests (no -x: the list of what differs).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-step}
OLD=$GRAFT_REPO_ROOT/cnn_graph_amd/libcheb_old.so
mkdir -p $OUT
for i in 1 2; do
for v in new old; do
if [ $v = old ]; then export CG_LIB_PATH=$OLD; else unset CG_LIB_PATH; fi
timeout -k 10 300 python bench.py --config E --no-cpu-baseline > $OUT/E.$v.$i.json 2>$OUT/E.err || { tail -20 $OUT/E.err; exit 1; }
timeout -k 10 300 python scripts/bench_configs.py E > $OUT/L.$v.$i.json 2>$OUT/L.err || { tail -20 $OUT/L.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/E.$v.$i.json'));print('$v E', d['value'], d['ms_per_step'])"
tail -1 $OUT/L.$v.$i.json
done
done
unset CG_LIB_PATH
timeout -k 10 600 python -u -m pytest tests/test_gpu_lstm.py -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1; echo "pytest rc=$?"
tail -15 $OUT/pytest.txt
