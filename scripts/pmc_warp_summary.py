#!/usr/bin/env python
"""Per-launch averages of the counters scripts/pmc_warp.sh collected for the 4K x 32 k_warp_diff
launches.  Usage: python scripts/pmc_warp_summary.py gpurun_out/pmc_warp"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
acc = collections.defaultdict(float)
n = collections.defaultdict(set)
for f in sorted(glob.glob(os.path.join(d, "*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if "k_warp_diff" not in r["Kernel_Name"] or int(r["Grid_Size"]) < 3840 * 2160 * 32 // 64:
            continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
        n[r["Counter_Name"]].add(r["Dispatch_Id"])
for k in sorted(acc):
    print(f"{k:24s} {acc[k] / max(1, len(n[k])):16.0f}  ({len(n[k])} launches)")
