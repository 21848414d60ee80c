#!/bin/bash
# LDS bank-conflict attribution of cheb_fwd_fast (config B, orders layout) on the
# debug build: one rocprofv3 PMC pass per ablation flag set.  bash scripts/gpu_r04_lds.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${1:-r04_lds}
mkdir -p $O
for F in 0 2 6 70 134 198 16; do
  timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS -d $O/f$F -o pmc --output-format csv -- python3 scripts/lds_attrib.py $F > $O/f$F.log 2>&1 || { echo "PMC_FAIL $F"; tail -20 $O/f$F.log; exit 1; }
done
python3 - <<PY
import csv, glob, json
out = {}
for d in sorted(glob.glob("$O/f*/")):
    f = d.rstrip("/").split("/")[-1]
    rows = [r for p in glob.glob(d + "**/*counter_collection.csv", recursive=True) for r in csv.DictReader(open(p))]
    acc = {}
    for r in rows:
        if "cheb_fwd_fast" not in r.get("Kernel_Name", ""):
            continue
        acc.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    out[f] = {k: sum(v) / len(v) for k, v in acc.items()}
    c = out[f]
    if c.get("SQ_LDS_IDX_ACTIVE"):
        c["conflict_frac"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
print(json.dumps(out, indent=1))
json.dump(out, open("$O/lds_attrib.json", "w"), indent=1)
PY
echo DONE
