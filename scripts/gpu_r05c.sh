#!/bin/bash
# bisect the LSTM failure over experiment libs; forward A/B bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05c}
mkdir -p $OUT
T="tests/test_gpu_lstm.py::test_two_layer_static_rnn_vs_oracle tests/test_gpu_lstm.py::test_config_E_sequence_path_equals_cell_steps"
for L in cur e00 e10 e01; do
  if [ $L == cur ]; then LP=""; else LP="scripts/ablib/libcheb_$L.so"; fi
  CG_LIB_PATH=$LP timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread $T > $OUT/t_$L.txt 2>&1
  echo "$L: $(tail -1 $OUT/t_$L.txt)"
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 400 --warmup 40 --no-cpu-baseline > $OUT/bench_new$i.json 2>&1 || { echo BENCH_FAIL; tail -20 $OUT/bench_new$i.json; exit 1; }
  CG_LIB_PATH=scripts/ablib/libcheb_base.so timeout -k 10 300 python bench.py --steps 400 --warmup 40 --no-cpu-baseline > $OUT/bench_base$i.json 2>&1 || { echo BENCHB_FAIL; tail -20 $OUT/bench_base$i.json; exit 1; }
done
python3 - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/r05c/bench_*.json')):
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split('/')[-1], d['value'], d['ms_per_step'], d['kernels']['fwd']['avg_ms'], d['kernels']['bwd']['avg_ms'])
PY
