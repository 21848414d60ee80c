#!/bin/bash
# r03: every -m gpu test, then config timings (C1 C2 D(N=256) E E_step R) and
# kernel traces of D(N=256) and E.   bash scripts/gpu_r03_full.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-r03_full}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --tb=short --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1; rc=$?
grep -E "FAIL|Error|passed|failed" $O/pytest_gpu.txt | tail -30
[ $rc -eq 0 ] || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 600 python3 scripts/bench_configs.py C1 C2 E E_step R > $O/configs.jsonl 2> $O/configs.err && cat $O/configs.jsonl &&
timeout -k 10 400 python3 scripts/bench_configs.py D --d-batch 256 > $O/D256.jsonl 2> $O/D256.err && cat $O/D256.jsonl &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/ktD -o kt --output-format csv -- python3 scripts/bench_configs.py D --d-batch 256 --rounds 1 > $O/ktD.log 2>&1 && echo KTD_OK &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ktE -o kt --output-format csv -- python3 scripts/bench_configs.py E > $O/ktE.log 2>&1 && echo KTE_OK &&
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY -d $O/pmcE -o pmc --output-format csv -- python3 scripts/bench_configs.py E --rounds 1 > $O/pmcE.log 2>&1 && echo PMCE_OK &&
python3 scripts/pmc_table.py $O/ktE > $O/tableE.json && python3 scripts/pmc_table.py $O/pmcE > $O/tableE_pmc.json && python3 scripts/pmc_table.py $O/ktD > $O/tableD.json && echo TABLES_OK
