#!/usr/bin/env python3
"""Top kernels of a rocprofv3 --kernel-trace --stats output directory:
   python3 scripts/kt_top.py DIR [n]"""
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/kt_kernel_stats.csv", recursive=True)[0]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
for i, r in enumerate(csv.DictReader(open(f))):
    if i < n:
        print(f"{r['Name'][:70]:70s} {r['Calls']:>6s} {float(r['AverageNs']) / 1e3:9.2f} us "
              f"{float(r['Percentage']):6.2f} %")
