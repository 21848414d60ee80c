#!/bin/bash
# rocprofv3 passes over the bench (kernel trace + stats, then PMC counters in
# SEPARATE passes as MI355X_MICROARCH.md prescribes; never combined with
# sys/runtime traces).  Summary: gpurun_out/$TAG/summary.json (copy it to
# profiles/pmc_latest.json to let bench.py report roofline.traffic).
#   bash scripts/prof_pmc.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-prof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
BENCH="bench.py --steps 50 --warmup 10 --no-cpu-baseline --graph off"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 $BENCH > $OUT/kt.log 2>&1 || { echo KT_FAIL; tail -20 $OUT/kt.log; exit 1; }
for C in FETCH_SIZE WRITE_SIZE "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS" "TCC_HIT_sum TCC_MISS_sum" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  N=$(echo $C | tr ' ' '_')
  timeout -s KILL 150 rocprofv3 --pmc $C -d $OUT/pmc_$N -o pmc --output-format csv -- python3 $BENCH > $OUT/pmc_$N.log 2>&1 || { echo "PMC_FAIL $C"; tail -20 $OUT/pmc_$N.log; exit 1; }
done
python3 scripts/pmc_summary.py $OUT $TAG > $OUT/summary.json 2>&1
cat $OUT/summary.json
