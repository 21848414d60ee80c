#!/bin/bash
# LSTM + group tests, configs E and R timing, BPTT-step ablation stamps (debug build)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05g}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_lstm.py tests/test_gpu_group.py > $OUT/pytest.txt 2>&1 || { echo TEST_FAIL; tail -60 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
timeout -k 10 300 python scripts/bench_configs.py E R E R --no-cpu > $OUT/cfg.jsonl 2>&1 || { echo CFG_FAIL; tail -20 $OUT/cfg.jsonl; exit 1; }
cat $OUT/cfg.jsonl
CG_LIB_PATH=scripts/ablib/dbg.so timeout -k 10 200 python scripts/ablate_bstep.py > $OUT/ablate_bstep.json 2> $OUT/ablate_bstep.err || { echo ABL_FAIL; tail -20 $OUT/ablate_bstep.err; exit 1; }
python3 -c "
import json
for k,v in json.load(open('$OUT/ablate_bstep.json')).items(): print(k, v)
"
