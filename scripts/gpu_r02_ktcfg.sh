# r02: rocprofv3 kernel traces of configs C2 and D (rows and planes basis
# layouts) and E with the final library
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02_final4/ktcfg
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rows -o cfg --output-format csv -- python3 scripts/bench_configs.py C2 D E > $O/rows.jsonl 2> $O/rows.err && echo ROWS_OK &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/planes -o cfg --output-format csv -- python3 scripts/bench_configs.py C2 D --layout planes > $O/planes.jsonl 2> $O/planes.err && echo PLANES_OK
