#!/usr/bin/env python
"""Per-level LK kernel durations (us) from a rocprofv3 kernel-trace CSV, averaged over steps.

Levels are recovered from dispatch order: within a step the LK kernels run maxLevel..0.
Usage: python scripts/lk_levels.py <run_kernel_trace.csv>
"""
import csv
import sys
from collections import defaultdict


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    per = defaultdict(list)
    lvl = {}
    for r in rows:
        name = (r.get("Kernel_Name") or r.get("Name")).split("(")[0]
        if "k_gray_pad" in name:
            lvl.clear()
        for key in ("k_lk_class", "k_lk_A", "k_lk_iter", "k_lk_level"):
            if key in name:
                n = lvl.get(key, 0)
                lvl[key] = n + 1
                dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                per[(key, n)].append(dur)
    for (key, n), v in sorted(per.items()):
        print(f"{key:12s} dispatch#{n} (level maxL-{n}): avg {sum(v)/len(v):8.1f} us over {len(v)}")


if __name__ == "__main__":
    main()
