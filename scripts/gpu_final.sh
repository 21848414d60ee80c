#!/bin/bash
# End-of-round GPU pass: smoke, every -m gpu test, the bench line (with the
# CPU baseline), the other configurations' timings (A, C1, C2, D, E, R with
# their CPU legs; bench.py --config D / E lines), kernel traces of configs A
# and E, and the bench's rocprofv3 kernel trace + PMC passes (prof_pmc.sh:
# FETCH_SIZE and WRITE_SIZE in separate runs).  Stops at the first failing
# step.   bash scripts/gpu_final.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo SMOKE_FAIL; tail -30 $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.txt | cut -c1-300; exit 1; }
tail -1 $OUT/pytest_gpu.txt
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 10 > $OUT/bench.json 2>$OUT/bench.err || { echo BENCH_FAIL; tail -30 $OUT/bench.err; exit 1; }
tail -1 $OUT/bench.json | cut -c1-300
timeout -k 10 300 python bench.py --config E --steps 30 --warmup 3 --cpu-seconds 8 > $OUT/bench_E.json 2>$OUT/bench_E.err || { echo BENCHE_FAIL; tail -30 $OUT/bench_E.err; exit 1; }
timeout -k 10 400 python bench.py --config D --steps 5 --warmup 1 --cpu-seconds 8 > $OUT/bench_D.json 2>$OUT/bench_D.err || { echo BENCHD_FAIL; tail -30 $OUT/bench_D.err; exit 1; }
timeout -k 10 700 python scripts/bench_configs.py A C1 C2 D E R > $OUT/configs.jsonl 2>$OUT/configs.err || { echo CFG_FAIL; tail -20 $OUT/configs.err; exit 1; }
grep config $OUT/configs.jsonl | cut -c1-250
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/ktA -o A --output-format csv -- python3 scripts/bench_configs.py A --no-cpu > $OUT/ktA.log 2>&1 || { echo KTA_FAIL; tail -20 $OUT/ktA.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/ktE -o E --output-format csv -- python3 scripts/bench_configs.py E --no-cpu > $OUT/ktE.log 2>&1 || { echo KTE_FAIL; tail -20 $OUT/ktE.log; exit 1; }
bash scripts/prof_pmc.sh $TAG/pmc > $OUT/pmc.log 2>&1 || { echo PMC_FAIL; tail -20 $OUT/pmc.log; exit 1; }
tail -5 $OUT/pmc.log
