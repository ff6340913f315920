"""Summarize scripts/warp_burst.sh's output (gpurun_out/burst) per launch of the burst.

Columns per k_warp_diff launch (launch order): duration by kernel records; with counters on, the
dispatch's duration, GRBM_GUI_ACTIVE / 8 / duration (the effective clock, MI355X_MICROARCH.md DVFS
note; it reads high below ~0.3 ms dispatches, so only its trend counts) and SQ_BUSY_CYCLES; from the
stamped build, the in-kernel clock and the median workgroup cycles.
Usage: python scripts/warp_burst_summary.py gpurun_out/burst > profiles/r06_warp_burst.txt
"""
import collections
import csv
import glob
import json
import os
import sys


def kt_durations(d, name):
    f = glob.glob(os.path.join(d, "**", "run_kernel_trace.csv"), recursive=True)
    if not f:
        return {}
    rows = [r for r in csv.DictReader(open(f[0])) if name in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return {int(r["Dispatch_Id"]): (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows}


def counters(d):
    f = glob.glob(os.path.join(d, "**", "run_counter_collection.csv"), recursive=True)
    out = collections.defaultdict(dict)
    if not f:
        return out
    for r in csv.DictReader(open(f[0])):
        if "k_warp_diff" not in r["Kernel_Name"]:
            continue
        out[int(r["Dispatch_Id"])][r["Counter_Name"]] = out[int(r["Dispatch_Id"])].get(r["Counter_Name"], 0.0) + \
            float(r["Counter_Value"])
    return out


def blocks(vals, n=10):
    """Means over consecutive blocks of n launches."""
    return [round(sum(vals[i:i + n]) / len(vals[i:i + n]), 1) for i in range(0, len(vals), n)]


def main():
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/burst"
    print("# k_warp_diff (4K gray x 32, affine true H) burst of 300 launches after 2 s idle, per launch in order;")
    print("# means over blocks of 10 consecutive launches (the first launch is the one before the idle).")
    kt = kt_durations(os.path.join(d, "kt"), "k_warp_diff")
    v = [kt[k] for k in sorted(kt)]
    print(f"kernel records, us ({len(v)}):            {blocks(v)}")
    probe = kt_durations(os.path.join(d, "probe"), "k_stream3")
    pv = [probe[k] for k in sorted(probe)]
    print(f"copy probe k_stream3 records, us ({len(pv)}): {blocks(pv)}")
    pk = kt_durations(os.path.join(d, "pmc"), "k_warp_diff")
    pc = counters(os.path.join(d, "pmc"))
    ids = [k for k in sorted(pk) if k in pc]
    if ids:
        dur = [pk[k] for k in ids]
        clk = [pc[k].get("GRBM_GUI_ACTIVE", 0) / 8 / (pk[k] * 1e-6) / 1e6 for k in ids]
        busy = [pc[k].get("SQ_BUSY_CYCLES", 0) / 1e3 for k in ids]
        print(f"with counters: records, us ({len(dur)}):   {blocks(dur)}")
        print(f"  GRBM_GUI_ACTIVE/8/duration, MHz:          {blocks(clk)}")
        print(f"  SQ_BUSY_CYCLES per dispatch, thousands:   {blocks(busy)}")
    sf = os.path.join(d, "stamp.json")
    if os.path.exists(sf):
        s = json.loads(open(sf).read().strip().splitlines()[-1])
        rows = s.get("stamps", {}).get("rows", [])
        if rows:
            print(f"stamped build (no profiler), wall {s['wall_us_per_launch']} us per launch:")
            print(f"  in-kernel clock, MHz:                     {blocks([r[1] for r in rows])}")
            print(f"  median workgroup cycles, thousands:       {blocks([r[2] / 1e3 for r in rows])}")
            print(f"  launch span of the sampled workgroups, us: {blocks([r[3] for r in rows])}")


if __name__ == "__main__":
    main()
