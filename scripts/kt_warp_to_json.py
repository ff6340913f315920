"""Turn a rocprofv3 --kernel-trace run of `bench.py --only-roofline` into profiles/warp_kernel_trace.json:
the average kernel-record duration of the roofline leg's launches (k_warp_prep + k_warp_diff) and of
the copy-ceiling probe (k_stream3), and the fractions of the 8 TB/s peak they give for the 3 B/px
algorithmic bytes.
bench.py attaches it as roofline.kernel_trace when its src_sha256 matches the loaded library.
Usage: python scripts/kt_warp_to_json.py gpurun_out/r04/warp_kt 3840x2160x32 [out.json] [timed]
timed: average only the last `timed` launches of each kernel (the leg's timed launches; the ones
before are its warmup, bench.py --roofline-warmup).
"""
import csv
import glob
import json
import os
import sys

HBM_PEAK_GBS = 8000.0


def bench_stamp(d):
    for f in sorted(glob.glob(os.path.join(d, "*.json"))):
        for line in open(f):
            line = line.strip()
            if line.startswith("{"):
                try:
                    return json.loads(line)["build"]["src_sha256"]
                except (ValueError, KeyError, TypeError):
                    pass
    return None


d, config = sys.argv[1], sys.argv[2]
timed = int(sys.argv[4]) if len(sys.argv) > 4 else 0
out = sys.argv[3] if len(sys.argv) > 3 and sys.argv[3] != "-" else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                         "warp_kernel_trace.json")
w, h, b = (int(v) for v in config.split("x"))
alg = 3.0 * w * h * b
dur = {"k_warp_diff": [], "k_stream3": [], "k_warp_prep": []}
prep_threads = ((w // 128) * (h // 64) // 32) * 256 * b        # k_warp_prep of this launch size
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        threads = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        for k in dur:
            # the roofline launches are the large grids (k_warp_diff: w*h*b/32 threads; k_stream3: /16)
            big = threads >= prep_threads if k == "k_warp_prep" else threads >= (w * h * b) // 64
            if k in name and big:
                dur[k].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
for k in dur:
    dur[k] = [x for _, x in sorted(dur[k])]
    if timed:
        dur[k] = dur[k][-timed:]
res = dict(config=config, algorithmic_bytes_per_launch=int(alg), source=os.path.basename(os.path.normpath(d)),
           src_sha256=bench_stamp(d), averaged=f"last {timed} launches per kernel" if timed else "all launches")
for k, v in dur.items():
    if not v:
        continue
    ns = sum(v) / len(v)
    res[k] = dict(launches=len(v), avg_us=round(ns / 1e3, 2), min_us=round(min(v) / 1e3, 2),
                  achieved_gbs=round(alg / ns, 1), frac=round(alg / ns / HBM_PEAK_GBS, 4))
if "k_warp_diff" in res and "k_warp_prep" in res:
    # the launch is the prep kernel + k_warp_diff back to back on one stream: both count
    ns = (res["k_warp_diff"]["avg_us"] + res["k_warp_prep"]["avg_us"]) * 1e3
    res["launch"] = dict(avg_us=round(ns / 1e3, 2), achieved_gbs=round(alg / ns, 1), frac=round(alg / ns / HBM_PEAK_GBS, 4),
                         what="k_warp_prep + k_warp_diff average kernel records")
if "k_stream3" in res and ("launch" in res or "k_warp_diff" in res):
    lu = res["launch"]["avg_us"] if "launch" in res else res["k_warp_diff"]["avg_us"]
    res["frac_of_copy_ceiling"] = round(res["k_stream3"]["avg_us"] / lu, 4)
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
