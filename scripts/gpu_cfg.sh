set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/cfg1
timeout -k 10 400 python scripts/bench_configs.py > gpurun_out/cfg1/cfg.log 2>&1 || { tail -20 gpurun_out/cfg1/cfg.log; exit 1; }
grep config gpurun_out/cfg1/cfg.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/cfg1/prof -o kt --output-format csv -- python3 scripts/bench_configs.py C1 C2 D > gpurun_out/cfg1/prof.log 2>&1 || { tail -20 gpurun_out/cfg1/prof.log; exit 1; }
find gpurun_out/cfg1/prof -name "*kernel_stats.csv" -exec cut -c1-200 {} \; | head -20
