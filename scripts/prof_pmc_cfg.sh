#!/bin/bash
# rocprofv3 kernel trace + PMC passes (each counter set in its own run, never
# with trace domains) over one bench_configs.py configuration, then the
# per-kernel table (scripts/pmc_table.py).   bash scripts/prof_pmc_cfg.sh TAG CFG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-pmc_cfg}
CFG=${2:-E}
OUT=gpurun_out/$TAG
mkdir -p $OUT
RUN="scripts/bench_configs.py $CFG --no-cpu"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o kt --output-format csv -- python3 $RUN > $OUT/kt.log 2>&1 || { echo KT_FAIL; tail -20 $OUT/kt.log; exit 1; }
for C in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "TCC_HIT_sum TCC_MISS_sum"; do
  N=$(echo $C | tr ' ' '_')
  timeout -s KILL 240 rocprofv3 --pmc $C -d $OUT/pmc_$N -o pmc --output-format csv -- python3 $RUN > $OUT/pmc_$N.log 2>&1 || { echo "PMC_FAIL $C"; tail -20 $OUT/pmc_$N.log; exit 1; }
done
python3 scripts/pmc_table.py $OUT > $OUT/table.json 2>&1
head -c 3000 $OUT/table.json
