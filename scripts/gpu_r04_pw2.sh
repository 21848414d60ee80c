#!/bin/bash
# r04: paired CSR-metadata reads in every resident SpMM (group kernels, the
# gconv-LSTM kernels): tests, R and E bench lines.   bash scripts/gpu_r04_pw2.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_pw2}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_group.py tests/test_gpu_model.py tests/test_gpu_lstm.py > $O/pytest.txt 2>&1
rc=$?; tail -5 $O/pytest.txt; [ $rc -le 1 ] || exit 1
for rep in 1 2; do
  timeout -k 10 300 python3 scripts/bench_configs.py R E --no-cpu >> $O/RE.jsonl 2>> $O/RE.err || { tail -5 $O/RE.err; exit 1; }
done
cut -c1-250 $O/RE.jsonl
timeout -k 10 200 python3 scripts/stamps_R.py > $O/stampsR.json 2>> $O/RE.err || { tail -5 $O/RE.err; exit 1; }
timeout -k 10 200 python3 scripts/stamps_E.py > $O/stampsE.json 2>> $O/RE.err || { tail -5 $O/RE.err; exit 1; }
cut -c1-300 $O/stampsR.json; cat $O/stampsE.json
echo DONE
