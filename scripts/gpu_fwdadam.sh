#!/bin/bash
# Adam-in-forward (cg_cheb_forward_adam): its GPU tests, then the exchange-step
# bench at N = 1 (--force-allreduce: RCCL all-reduce over one rank) with the
# update in the next forward vs the separate k_adam launch, same box.
#   bash scripts/gpu_fwdadam.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-fwdadam}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused_adam.py tests/test_gpu_basis_layout.py > $OUT/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for r in 1 2; do
  for mode in "" "--unfused-adam"; do
    timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --force-allreduce $mode > $OUT/b.json 2>$OUT/b.err || { echo BENCH_FAIL; tail -20 $OUT/b.err; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/b.json') if l.startswith('{')][-1]); print('${mode:-fwd_adam}', d['value'], d['ms_per_step'], d['config']['adam'])" | tee -a $OUT/summary.txt
  done
done
