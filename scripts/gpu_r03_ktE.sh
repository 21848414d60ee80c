#!/bin/bash
# r03: kernel trace of config E (fwd+bwd) + per-kernel table
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
TAG=${1:-r03_ktE}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ktE -o kt --output-format csv -- python3 scripts/bench_configs.py E > $O/ktE.log 2>&1 && echo KTE_OK &&
python3 scripts/pmc_table.py $O/ktE > $O/tableE.json && cat $O/tableE.json | head -c 3000
