#!/usr/bin/env python3
"""Per-kernel table of a rocprofv3 output tree: average duration (kernel
trace stats) and per-dispatch averages of every PMC counter, with the
derived quantities the bench and DESIGN.md quote:
  fetch_bytes_x2  FETCH_SIZE (KB) x 1024 x 2  (gfx950: FETCH_SIZE counts half
                  the bytes of wide reads, MI355X_MICROARCH.md §HBM)
  write_bytes     WRITE_SIZE (KB) x 1024
  l2_hit          TCC_HIT / (TCC_HIT + TCC_MISS)
  mfma_busy_us    SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x 2.4 GHz): the MFMA
                  pipe time per SIMD (the counter sums the busy cycles of
                  every MFMA instruction chip-wide)
  mfma_busy_frac  mfma_busy_us / the kernel's average duration
Usage: python scripts/pmc_table.py ROOT [--grid-filter SUBSTR] > table.json"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

SIMDS, CLK = 1024, 2.4e9


def short(name):
    m = re.search(r"(cheb_\w+|k_\w+|__amd\w+)", name)
    return m.group(1) if m else name[:40]


def main(root):
    kern = defaultdict(lambda: {"calls": 0, "total_ns": 0.0})
    for f in glob.glob(os.path.join(root, "**", "*kernel_stats.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = short(row["Name"])
            kern[k]["calls"] += int(row["Calls"])
            kern[k]["total_ns"] += float(row["TotalDurationNs"])
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            acc[(short(row["Kernel_Name"]), row["Counter_Name"])].append(float(row["Counter_Value"]))
    out = {}
    for k, v in kern.items():
        if k.startswith("k_") or k.startswith("cheb"):
            out[k] = {"calls": v["calls"], "avg_us": round(v["total_ns"] / v["calls"] / 1e3, 3)}
    for (k, cn), vals in acc.items():
        if not (k.startswith("k_") or k.startswith("cheb")):
            continue
        out.setdefault(k, {})[cn] = round(sum(vals) / len(vals), 1)
    for k, c in out.items():
        if "FETCH_SIZE" in c:
            c["fetch_bytes_x2"] = int(c["FETCH_SIZE"] * 2048)
        if "WRITE_SIZE" in c:
            c["write_bytes"] = int(c["WRITE_SIZE"] * 1024)
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c:
            c["l2_hit"] = round(c["TCC_HIT_sum"] / max(1.0, c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 4)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            c["mfma_busy_us"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / SIMDS / CLK * 1e6, 3)
            if "avg_us" in c:
                c["mfma_busy_frac"] = round(c["mfma_busy_us"] / c["avg_us"], 4)
    print(json.dumps({"source": root, "kernels": out}, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1])
