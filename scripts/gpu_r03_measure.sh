#!/bin/bash
# r03: config D at its per-rank workload (N = 256 = 2048 / 8), kernel trace and
# PMC passes (FETCH / WRITE / TCC hit-miss / MFMA busy, each its own run), and
# the MFMA-busy pass of the headline bench (cheb_fwd_fast's contraction).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-r03_measure}
O=gpurun_out/$TAG
mkdir -p $O
CFG="scripts/bench_configs.py D --d-batch 256"
timeout -k 10 400 python3 $CFG > $O/D256_rows.jsonl 2> $O/D256_rows.err && echo D_ROWS_OK && cat $O/D256_rows.jsonl &&
timeout -k 10 400 python3 $CFG --layout planes > $O/D256_planes.jsonl 2> $O/D256_planes.err && echo D_PLANES_OK && cat $O/D256_planes.jsonl &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/ktD -o kt --output-format csv -- python3 $CFG --rounds 1 > $O/ktD.log 2>&1 && echo KT_OK &&
for C in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY"; do
  N=$(echo $C | tr ' ' '_')
  timeout -k 10 400 rocprofv3 --pmc $C -d $O/pmcD_$N -o pmc --output-format csv -- python3 $CFG --rounds 1 > $O/pmcD_$N.log 2>&1 || { echo "PMC_FAIL $C"; tail -20 $O/pmcD_$N.log; exit 1; }
  echo "PMC_OK $C"
done &&
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmcB_mfma -o pmc --output-format csv -- python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline > $O/pmcB_mfma.log 2>&1 && echo PMCB_OK
