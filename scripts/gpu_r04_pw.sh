#!/bin/bash
# r04: paired CSR-metadata reads in k_grp16_fwd (CG_SPMM_PW=1/0): group tests,
# config R A/B, forward stamps.   bash scripts/gpu_r04_pw.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_pw}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_group.py tests/test_gpu_model.py > $O/pytest.txt 2>&1
rc=$?; tail -5 $O/pytest.txt; [ $rc -le 1 ] || exit 1
for rep in 1 2; do
  for v in 1 0; do
    CG_SPMM_PW=$v timeout -k 10 200 python3 scripts/bench_configs.py R --no-cpu >> $O/R_pw$v.jsonl 2>> $O/R.err || { tail -5 $O/R.err; exit 1; }
  done
done
for v in 1 0; do echo "== CG_SPMM_PW=$v"; cut -c1-250 $O/R_pw$v.jsonl; done
for v in 1 0; do
  CG_SPMM_PW=$v timeout -k 10 200 python3 scripts/stamps_R.py >> $O/stampsR.jsonl 2>> $O/R.err || { tail -5 $O/R.err; exit 1; }
done
cut -c1-200 $O/stampsR.jsonl
echo DONE
