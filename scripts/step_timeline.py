#!/usr/bin/env python
"""Timeline of one pipeline step from a rocprofv3 --kernel-trace CSV: every kernel of the LAST step
(the kernels from the last k_front launch of a frame-mode front end to the last k_warp_diff), with
its start and end relative to the step's first kernel, in microseconds.

Usage: python scripts/step_timeline.py <run_kernel_trace.csv> [first-kernel substring]
"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    first = sys.argv[2] if len(sys.argv) > 2 else "k_front<4, 0"
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    name = lambda r: (r.get("Kernel_Name") or r.get("Name")).split("(")[0].replace("void ", "").replace("mdx::", "")
    starts = [i for i, r in enumerate(rows) if first in name(r)]
    # a step starts at a frame-mode k_front of the first frames; take the last complete step
    i0 = starts[-2] if len(starts) >= 2 else starts[-1]
    seg = [r for r in rows[i0:] if "copyBuffer" not in name(r)]
    ends = [j for j, r in enumerate(seg) if "k_warp_diff" in name(r)]
    seg = seg[:ends[0] + 1] if ends else seg
    t0 = int(seg[0]["Start_Timestamp"])
    for r in seg:
        s, e = (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3
        g = f"{r.get('Grid_Size_X', '')}x{r.get('Grid_Size_Y', '')}x{r.get('Grid_Size_Z', '')}"
        print(f"{s:9.1f} {e:9.1f} {e - s:8.1f}  {name(r)} {g}")


if __name__ == "__main__":
    main()
