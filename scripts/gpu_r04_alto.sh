#!/bin/bash
# r04: config R with k_grp16_fwd's two waves per SIMD in opposite MFMA / SpMM phase order
# (scripts/dbg/libcheb_alt_o.so) vs one order (default library), alternating.
#   bash scripts/gpu_r04_alto.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_alto}
mkdir -p $O
for rep in 1 2; do
  for v in def alt_o; do
    if [ $v = def ]; then L=""; else L=$PWD/scripts/dbg/libcheb_$v.so; fi
    CG_LIB_PATH=$L timeout -k 10 200 python3 scripts/bench_configs.py R --no-cpu > $O/tmp.json 2>> $O/R.err || { tail -5 $O/R.err; exit 1; }
    echo "$v $(cut -c1-250 $O/tmp.json)" >> $O/R_ab.txt
  done
done
cat $O/R_ab.txt
echo DONE
