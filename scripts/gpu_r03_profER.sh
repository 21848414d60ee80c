#!/bin/bash
# Kernel traces and PMC passes (separate runs) of configs E (gconv-LSTM) and R (ResGNN step)
#   bash scripts/gpu_r03_profER.sh TAG [CONFIGS]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_profER}
mkdir -p $O
for CF in ${2:-E R}; do
  D=$O/$CF
  mkdir -p $D
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/kt -o kt --output-format csv -- python3 scripts/bench_configs.py $CF --rounds 1 > $D/kt.log 2>&1 || { echo KT_FAIL $CF; tail -20 $D/kt.log; exit 1; }
  for C in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAIT_INST_LDS" FETCH_SIZE WRITE_SIZE "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
    N=$(echo $C | cut -d' ' -f1)
    timeout -k 10 300 rocprofv3 --pmc $C -d $D/pmc_$N -o pmc --output-format csv -- python3 scripts/bench_configs.py $CF --rounds 1 > $D/pmc_$N.log 2>&1 || { echo "PMC_FAIL $CF $C"; tail -20 $D/pmc_$N.log; exit 1; }
  done
  python3 scripts/pmc_table.py $D > $O/table$CF.json 2>&1 || true
done
echo DONE
