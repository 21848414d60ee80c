#!/bin/bash
# r03: bench rows vs orders basis layout, alternating, same box
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-r03_layout}
O=gpurun_out/$TAG
mkdir -p $O
[ -n "$NOTEST" ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_basis_layout.py tests/test_gpu_parity.py tests/test_gpu_fused_adam.py -x -q --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -20 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for r in 1 2 3 4 5; do
for lay in rows orders; do
timeout -k 10 200 python3 bench.py --steps 400 --warmup 40 --no-cpu-baseline --basis-layout $lay > $O/bench_${lay}_$r.json 2> $O/bench_${lay}_$r.err || exit 1
python3 -c "
import json,sys; d=json.load(open('$O/bench_${lay}_$r.json'))
print('$lay', $r, d['value'], d['ms_per_step'], d['kernels']['fwd']['avg_ms'], d['kernels']['bwd']['avg_ms'], d['roofline_spmm_fwd']['frac'], d['roofline']['frac'])"
done
done
