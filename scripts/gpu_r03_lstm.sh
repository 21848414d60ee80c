#!/bin/bash
# r03: the one-launch gconv-LSTM layer forward + one-launch BPTT step:
# GPU tests, config E timings (seq / per-step / unfused), kernel trace + MFMA busy
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-r03_lstm}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_lstm.py -x -v --tb=short --timeout 200 --timeout-method thread > $O/pytest_lstm.txt 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error" $O/pytest_lstm.txt | tail -40
[ $rc -eq 0 ] || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 300 python3 scripts/bench_configs.py E E_step E_unfused > $O/configE.jsonl 2> $O/configE.err && cat $O/configE.jsonl &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ktE -o kt --output-format csv -- python3 scripts/bench_configs.py E > $O/ktE.log 2>&1 && echo KT_OK &&
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY -d $O/pmcE -o pmc --output-format csv -- python3 scripts/bench_configs.py E --rounds 1 > $O/pmcE.log 2>&1 && echo PMC_OK &&
python3 scripts/pmc_table.py $O > $O/table.json && echo TABLE_OK
