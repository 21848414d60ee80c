#!/bin/bash
# r04: the dW / train-op parity tests, the k_dw_direct A/B (CG_DW_DIRECT=1/0) on
# configs C2, E, R and D (planes, per-rank batch), then scripts/gpu_r04_grp.sh.
#   bash scripts/gpu_r04_ab.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_ab}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_dw_direct.py tests/test_gpu_train_ops.py tests/test_gpu_wide_fout.py > $O/pytest.txt 2>&1
rc=$?; tail -5 $O/pytest.txt; [ $rc -le 1 ] || exit 1
for rep in 1 2; do
  for v in 1 0; do
    CG_DW_DIRECT=$v timeout -k 10 300 python3 scripts/bench_configs.py C2 E R --no-cpu >> $O/ab_dw$v.jsonl 2>> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
  done
done
for v in 1 0; do
  CG_DW_DIRECT=$v timeout -k 10 300 python3 scripts/bench_configs.py D --d-batch 256 --layout planes --no-cpu >> $O/ab_dw$v.jsonl 2>> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
done
for v in 1 0; do echo "== CG_DW_DIRECT=$v"; cut -c1-230 $O/ab_dw$v.jsonl; done
bash scripts/gpu_r04_grp.sh ${1:-r04_ab}/grp
