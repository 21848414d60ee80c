#!/bin/bash
# r04: the LSTM tests, then config R's dW with the two-waves k_dw_direct forced (CG_DW_DIRECT=2) vs
# the default (k_dw_slabs below 1024 waves), plus E and R lines on the final tree.
#   bash scripts/gpu_r04_rdw.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_rdw}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_lstm.py > $O/pytest.txt 2>&1
rc=$?; tail -3 $O/pytest.txt; [ $rc -le 1 ] || exit 1
for rep in 1 2; do
  for v in 2 1; do
    CG_DW_DIRECT=$v timeout -k 10 200 python3 scripts/bench_configs.py R --no-cpu > $O/tmp.json 2>> $O/R.err || { tail -5 $O/R.err; exit 1; }
    echo "dw$v $(cut -c1-250 $O/tmp.json)" >> $O/R_ab.txt
  done
done
cat $O/R_ab.txt
timeout -k 10 200 python3 scripts/bench_configs.py E --no-cpu > $O/E.json 2>> $O/R.err || { tail -5 $O/R.err; exit 1; }
cut -c1-200 $O/E.json
echo DONE
