#!/bin/bash
# r03: 16-channel group kernels -- GPU tests touching the group path, then
# config R with the 16-channel and (CG_GRP16=0) 8-channel kernels, same box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-r03_grp}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_basis_layout.py tests/test_gpu_model.py tests/test_gpu_parity.py tests/test_gpu_filter.py -x -v --tb=short --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
grep -E "FAIL|Error|passed|failed" $O/pytest.txt | tail -20
[ $rc -eq 0 ] || { echo PYTEST_FAIL; exit 1; }
for r in 1 2; do
timeout -k 10 200 python3 scripts/bench_configs.py R > $O/R16_$r.jsonl 2>&1 && cat $O/R16_$r.jsonl &&
CG_GRP16=0 timeout -k 10 200 python3 scripts/bench_configs.py R > $O/R8_$r.jsonl 2>&1 && cat $O/R8_$r.jsonl || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ktR -o kt --output-format csv -- python3 scripts/bench_configs.py R > $O/ktR.log 2>&1 && echo KTR_OK &&
python3 scripts/pmc_table.py $O/ktR > $O/tableR.json
