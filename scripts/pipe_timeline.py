#!/usr/bin/env python
"""Timeline of one pipelined bench step from a rocprofv3 --kernel-trace CSV: the kernels between
the k_front (frame mode) launches that start steps `k` and `k + 1` (default: the 5th step seen),
with start / end relative to the first, in microseconds.

Usage: python scripts/pipe_timeline.py <run_kernel_trace.csv> [k]
"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    name = lambda r: (r.get("Kernel_Name") or r.get("Name")).split("(")[0].replace("void ", "").replace("mdx::", "")
    idx = [i for i, r in enumerate(rows) if "k_front<4, 0" in name(r)]
    t0 = int(rows[idx[k]]["Start_Timestamp"])
    for r in rows[idx[k]:idx[k + 2]]:
        s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
        g = f"{r.get('Grid_Size_X', '')}x{r.get('Grid_Size_Y', '')}x{r.get('Grid_Size_Z', '')}"
        print(f"{s:9.1f} {e:9.1f} {e - s:8.1f}  {name(r)} {g}")


if __name__ == "__main__":
    main()
