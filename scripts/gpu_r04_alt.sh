#!/bin/bash
# r04: config E with the paired-row SpMM in both gconv-LSTM kernels (default
# library) vs not in the forward (alt_b) vs in neither (alt_c): alternating runs.
#   bash scripts/gpu_r04_alt.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_alt}
mkdir -p $O
for rep in 1 2 3; do
  for v in def alt_b alt_c; do
    if [ $v = def ]; then L=""; else L=$PWD/scripts/dbg/libcheb_$v.so; fi
    CG_LIB_PATH=$L timeout -k 10 200 python3 scripts/bench_configs.py E --no-cpu > $O/tmp.json 2>> $O/E.err || { tail -5 $O/E.err; exit 1; }
    echo "$v $(cut -c1-200 $O/tmp.json)" >> $O/E_ab.txt
  done
done
cat $O/E_ab.txt
echo DONE
