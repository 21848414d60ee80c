# r02: kernel trace of config R (ResGNN training step, humanflow shape)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/t4
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o R -- python3 scripts/bench_configs.py R > $O/R.jsonl 2> $O/R.err && echo TRACE_OK
