#!/bin/bash
# r03 iteration: LSTM + layout/model GPU tests, seq ablation, configs E / R
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-r03_iter}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_lstm.py tests/test_gpu_basis_layout.py tests/test_gpu_model.py -x -v --tb=short --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
grep -E "FAIL|Error|passed|failed" $O/pytest.txt | tail -20
[ $rc -eq 0 ] || { echo PYTEST_FAIL; exit 1; }
timeout -k 10 300 python3 scripts/ablate_lstm.py > $O/ablate_lstm.json 2> $O/ablate_lstm.err && cat $O/ablate_lstm.json &&
timeout -k 10 300 python3 scripts/bench_configs.py E R > $O/configs.jsonl 2> $O/configs.err && cat $O/configs.jsonl
[ -n "$KT" ] || exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ktE -o kt --output-format csv -- python3 scripts/bench_configs.py E > $O/ktE.log 2>&1 && echo KTE_OK &&
python3 scripts/pmc_table.py $O/ktE > $O/tableE.json && head -c 2500 $O/tableE.json
[ -n "$KTR" ] || exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ktR -o kt --output-format csv -- python3 scripts/bench_configs.py R > $O/ktR.log 2>&1 && echo KTR_OK &&
python3 scripts/pmc_table.py $O/ktR > $O/tableR.json
