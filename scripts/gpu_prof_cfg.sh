#!/bin/bash
# per-config rocprofv3 kernel stats of scripts/bench_configs.py
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-profcfg}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for C in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$C -o kt --output-format csv -- python3 scripts/bench_configs.py $C > $OUT/$C.log 2>&1 || { tail -20 $OUT/$C.log; exit 1; }
  grep config $OUT/$C.log
  find $OUT/$C -name "*kernel_stats.csv" -exec cut -c1-150 {} \; | grep -v "at::native" | head -12
done
