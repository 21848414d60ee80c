#!/bin/bash
# One build -> measure iteration on MI355X: the fast-path GPU tests, the bench
# with both basis layouts (same box), and the debug-build phase timeline.
#   bash scripts/gpu_iter.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-iter}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_basis_layout.py tests/test_gpu_fused_adam.py tests/test_gpu_parity.py > $OUT/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest.txt; exit 1; }
tail -1 $OUT/pytest.txt
for L in rows orders rows orders; do
  timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --basis-layout $L >> $OUT/bench_$L.json 2>$OUT/bench_$L.err || { echo BENCH_FAIL; tail -20 $OUT/bench_$L.err; exit 1; }
done
python3 - $OUT <<'PY'
import json, sys
for L in ("rows", "orders"):
    for line in open(f"{sys.argv[1]}/bench_{L}.json"):
        d = json.loads(line)
        k = d["kernels"]
        print(L, d["value"], d["ms_per_step"], "fwd", k["fwd"]["avg_ms"], "bwd", k["bwd"]["avg_ms"], "frac_fwd", d["roofline_spmm_fwd"]["frac"])
PY
if [ -f scripts/_debug/libcheb_mi355_debug.so ]; then
  timeout -k 10 200 python scripts/phase_ts.py > $OUT/phase_ts.json 2>&1 || { echo TS_FAIL; tail -20 $OUT/phase_ts.json; exit 1; }
  python3 - $OUT <<'PY'
import json, sys
t = open(f"{sys.argv[1]}/phase_ts.json").read(); d = json.loads(t[t.index("{"):])
for k, v in d.items():
    print(k, "kernel", v["kernel_us"], " ".join(f"{n}={m[0]}/{m[1]}" for n, m in v["phase_us_median_max"].items()))
PY
fi
