#!/usr/bin/env python
"""Summarise a rocprofv3 --kernel-trace CSV per (kernel, grid) -> markdown table.

Usage: python scripts/summarize_prof.py <run_kernel_trace.csv> [title]
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    title = sys.argv[2] if len(sys.argv) > 2 else path
    rows = list(csv.DictReader(open(path)))
    agg = defaultdict(list)
    for r in rows:
        name = r.get("Kernel_Name") or r.get("Name")
        grid = f"{r.get('Grid_Size_X', r.get('Grid_Size', '?'))}x{r.get('Grid_Size_Y', '')}x{r.get('Grid_Size_Z', '')}"
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        agg[(name.split("(")[0], grid, r.get("Workgroup_Size_X", ""))].append(dur)
    tot = sum(sum(v) for v in agg.values())
    print(f"### {title}\n")
    print("| kernel | grid (threads) | wg | calls | avg us | min us | total ms | % |")
    print("|---|---|---|---|---|---|---|---|")
    for (k, g, wg), v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"| {k} | {g} | {wg} | {len(v)} | {sum(v)/len(v):.2f} | {min(v):.2f} | {sum(v)/1e3:.3f} | {100*sum(v)/tot:.1f} |")


if __name__ == "__main__":
    main()
