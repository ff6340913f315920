#!/usr/bin/env python
"""The last N kernels of a rocprofv3 --kernel-trace CSV, in start order, with start / end / duration
(us, relative to the first of them) and grid -- a timeline of the end of a run (e.g. bench.py's
one-band C4 loop or the live leg's last callbacks).

Usage: python scripts/kt_tail.py <run_kernel_trace.csv> [N=60]
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 60
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
seg = rows[-n:]
t0 = int(seg[0]["Start_Timestamp"])
for r in seg:
    nm = (r.get("Kernel_Name") or r.get("Name")).split("(")[0].replace("void ", "").replace("mdx::", "")
    s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
    g = f"{r.get('Grid_Size_X', '')}x{r.get('Grid_Size_Y', '')}x{r.get('Grid_Size_Z', '')}"
    print(f"{s:9.1f} {e:9.1f} {e - s:8.1f}  {nm} {g}")
