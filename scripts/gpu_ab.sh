#!/bin/bash
# Scratch A/B of two library builds (rewritten per experiment): the default
# in-tree library against $NEW (CG_LIB_PATH), bitwise outputs, timings
# interleaved, kernel traces of both.   bash scripts/gpu_ab.sh TAG NEW.so
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-ab}
NEW=$GRAFT_REPO_ROOT/${2:-cnn_graph_amd/libcheb_h1.so}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 200 python scripts/ab_seq.py $OUT/old.npz > $OUT/t_old0.json 2>$OUT/err.txt || { echo OLD_FAIL; tail -20 $OUT/err.txt; exit 1; }
cat $OUT/t_old0.json
CG_LIB_PATH=$NEW timeout -k 10 200 python scripts/ab_seq.py $OUT/new.npz --cmp $OUT/old.npz > $OUT/t_new0.json 2>$OUT/err.txt || { echo NEW_FAIL; cat $OUT/t_new0.json; tail -20 $OUT/err.txt; exit 1; }
cat $OUT/t_new0.json
for i in 1 2; do
timeout -k 10 200 python scripts/ab_seq.py $OUT/o.npz > $OUT/t_old$i.json 2>$OUT/err.txt || { echo OLD_FAIL; exit 1; }
cat $OUT/t_old$i.json
CG_LIB_PATH=$NEW timeout -k 10 200 python scripts/ab_seq.py $OUT/n.npz > $OUT/t_new$i.json 2>$OUT/err.txt || { echo NEW_FAIL; exit 1; }
cat $OUT/t_new$i.json
done
CG_LIB_PATH=$NEW timeout -k 10 600 python -u -m pytest tests/test_gpu_lstm.py tests/test_gpu_glstm_dp.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest_new.txt 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_new.txt | cut -c1-300; exit 1; }
tail -1 $OUT/pytest_new.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/kto -o o --output-format csv -- python3 scripts/ab_seq.py $OUT/x.npz --reps 5 > $OUT/kto.log 2>&1 || { echo KTO_FAIL; tail -20 $OUT/kto.log; exit 1; }
CG_LIB_PATH=$NEW timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/ktn -o n --output-format csv -- python3 scripts/ab_seq.py $OUT/x.npz --reps 5 > $OUT/ktn.log 2>&1 || { echo KTN_FAIL; tail -20 $OUT/ktn.log; exit 1; }
python3 - <<EOF
import csv
for t in ("kto/o", "ktn/n"):
    for r in list(csv.DictReader(open("$OUT/" + t + "_kernel_stats.csv")))[:5]:
        print(t, r["Name"][:50], r["Calls"], r["AverageNs"])
EOF
