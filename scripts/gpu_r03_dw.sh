#!/bin/bash
# r03: k_dw_slabs with 8 waves per block vs 4 (CG_DW_WAVES), same box: tests
# that pin the slabs, then configs E / R / C2 / D(N=32) under both
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-r03_dw}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_lstm.py tests/test_gpu_basis_layout.py tests/test_gpu_model.py tests/test_gpu_large.py -x -v --tb=short --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?
grep -E "FAIL|Error|passed|failed" $O/pytest.txt | tail -20
[ $rc -eq 0 ] || { echo PYTEST_FAIL; exit 1; }
for r in 1 2; do
for wv in 8 4; do
CG_DW_WAVES=$wv timeout -k 10 300 python3 scripts/bench_configs.py E R C2 D > $O/cfg_w${wv}_$r.jsonl 2> $O/cfg_w${wv}_$r.err || exit 1
echo "waves $wv run $r"; cat $O/cfg_w${wv}_$r.jsonl
done
done
