#!/bin/bash
# End-of-round GPU pass: smoke, every -m gpu test, the bench line (with the
# CPU baseline), the streaming / LSTM config timings, and the rocprofv3 kernel
# trace + PMC passes of the bench (FETCH_SIZE and WRITE_SIZE in separate runs),
# the C2 / D filters in the planes basis layout and a kernel trace of config R.
# Stops at the first failing step.   bash scripts/gpu_final.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo SMOKE_FAIL; tail -30 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.txt; exit 1; }
tail -1 $OUT/pytest_gpu.txt
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 10 > $OUT/bench.json 2>&1 || { echo BENCH_FAIL; tail -30 $OUT/bench.json; exit 1; }
tail -1 $OUT/bench.json
timeout -k 10 600 python scripts/bench_configs.py A C1 C2 D E R > $OUT/configs.jsonl 2>&1 || { echo CFG_FAIL; tail -20 $OUT/configs.jsonl; exit 1; }
grep config $OUT/configs.jsonl
timeout -k 10 300 python scripts/bench_configs.py C2 D --layout planes > $OUT/configs_planes.jsonl 2>&1 || { echo CFG_PLANES_FAIL; tail -20 $OUT/configs_planes.jsonl; exit 1; }
grep config $OUT/configs_planes.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ktR -o R --output-format csv -- python3 scripts/bench_configs.py R > $OUT/ktR.log 2>&1 || { echo KTR_FAIL; tail -20 $OUT/ktR.log; exit 1; }
bash scripts/prof_pmc.sh $TAG/pmc > $OUT/pmc.log 2>&1 || { echo PMC_FAIL; tail -20 $OUT/pmc.log; exit 1; }
tail -5 $OUT/pmc.log
