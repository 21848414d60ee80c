#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output: per-kernel average duration (kernel trace)
and per-dispatch average of every PMC counter, for the cnn_graph_amd kernels.

FETCH_SIZE / WRITE_SIZE are reported in KB by rocprofv3.  On gfx950
FETCH_SIZE reads half the bytes of wide coalesced streams
(MI355X_MICROARCH.md §HBM); both the raw value and x2 are printed."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(cheb_\w+|k_\w+|__amd\w+)", name)
    return m.group(1) if m else name[:40]


def main(root, tag=None):
    # the bench configuration these passes ran (bench.py defaults: config B)
    layout = os.environ.get("CG_BENCH_LAYOUT", "orders")  # bench.py's default --basis-layout
    out = {"config": {"M": 976, "N": 256, "K": 25, "Fin": 1, "Fout": 32, "layout": layout},
           "source": f"rocprofv3 passes of `bench.py --steps 50 --warmup 10` ({tag or root})",
           "kernels": {}, "counters": {}}
    for f in glob.glob(os.path.join(root, "**", "*kernel_stats.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Name"])
                if k.startswith("cheb") or k.startswith("k_"):
                    out["kernels"][k] = {"calls": int(row["Calls"]),
                                         "avg_us": round(float(row["AverageNs"]) / 1e3, 3)}
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name") or row.get("Kernel-Name") or ""
                k = short(name)
                if not (k.startswith("cheb") or k.startswith("k_")):
                    continue
                cn = row.get("Counter_Name") or row.get("Counter-Name")
                cv = float(row.get("Counter_Value") or row.get("Counter-Value") or 0)
                acc[(k, cn)].append(cv)
    for (k, cn), vals in sorted(acc.items()):
        # one row per dispatch (values are already summed over XCDs/instances)
        out["counters"].setdefault(k, {})[cn] = round(sum(vals) / len(vals), 1)
    for k, c in out["counters"].items():
        if "FETCH_SIZE" in c:
            c["FETCH_SIZE_x2_bytes"] = c["FETCH_SIZE"] * 1024 * 2
        if "WRITE_SIZE" in c:
            c["WRITE_SIZE_bytes"] = c["WRITE_SIZE"] * 1024
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            # summed over the 1024 SIMDs, shader clock 2.4 GHz: busy us of one SIMD
            c["mfma_busy_us"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * 2.4e3), 3)
            if k in out["kernels"]:
                c["mfma_busy_frac"] = round(c["mfma_busy_us"] / out["kernels"][k]["avg_us"], 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out", sys.argv[2] if len(sys.argv) > 2 else None)
