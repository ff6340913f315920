"""Summarise rocprofv3 --pmc CSVs (counter_collection) per kernel: mean counter value per dispatch.
Usage: python scripts/pmc_summary.py <dir> [kernel-substring]"""
import csv, glob, sys
from collections import defaultdict
d = sys.argv[1]; ks = sys.argv[2] if len(sys.argv) > 2 else "k_warp_diff"
vals = defaultdict(list)
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if ks in r.get("Kernel_Name", ""):
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(vals):
    v = vals[k]
    print(f"{k:28s} {sum(v)/len(v):16.1f}  (n={len(v)})")
