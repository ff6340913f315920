"""Summarize scripts/lk_probe.sh output: per-kernel avg duration and summed counters per launch."""
import collections, csv, glob, os, sys

d = sys.argv[1]
tfile = os.path.join(d, "stats", "run_kernel_trace.csv")
if not os.path.exists(tfile):
    tfile = sorted(glob.glob(os.path.join(d, "*", "run_kernel_trace.csv")))[0]
trace = list(csv.DictReader(open(tfile)))
dur = collections.defaultdict(list)
for r in trace:
    dur[r["Kernel_Name"].split("(")[0]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
ctr = collections.defaultdict(lambda: collections.defaultdict(float))
launches = collections.defaultdict(set)
for f in glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0]
        ctr[k][r["Counter_Name"]] += float(r["Counter_Value"])
        launches[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
for k in sorted(dur, key=lambda k: -sum(dur[k])):
    v = dur[k]
    print(f"{k:40s} n={len(v):4d} avg={sum(v)/len(v):9.1f}us total={sum(v)/1e3:8.2f}ms")
    for c, x in sorted(ctr[k].items()):
        n = len(launches[(k, c)])
        print(f"    {c:32s} per-launch {x / max(n, 1):16.1f}")
