"""Turn a scripts/pmc_sets.sh run (FETCH_SIZE / WRITE_SIZE passes over `bench.py --only-roofline`)
into profiles/pmc_warp_diff.json, the per-launch HBM traffic bench.py reports as roofline.traffic.

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half the bytes of a wide
streaming read, so read bytes = 2 * FETCH_SIZE KiB; WRITE_SIZE is exact.
Usage: python scripts/pmc_to_json.py gpurun_out/pmc_<tag> 3840x2160x32 [out.json]
"""
import collections
import csv
import glob
import json
import os
import sys


def bench_stamp(d):
    """src_sha256 of the library the profiled bench ran (its JSON line's build stamp, p1.json)."""
    for f in sorted(glob.glob(os.path.join(d, "p*.json"))):
        for line in open(f):
            line = line.strip()
            if line.startswith("{"):
                try:
                    return json.loads(line)["build"]["src_sha256"]
                except (ValueError, KeyError, TypeError):
                    pass
    return None

d, config = sys.argv[1], sys.argv[2]
out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(__file__), "..", "profiles", "pmc_warp_diff.json")
w, h, b = (int(v) for v in config.split("x"))
vals = collections.defaultdict(list)
prep = collections.defaultdict(list)
prep_threads = ((w // 128) * (h // 64) // 32) * 256 * b        # k_warp_prep of this launch size
for f in glob.glob(os.path.join(d, "*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        # the roofline launches are the large grids (w*h*b/32 threads: 128x64 tiles of 256 threads),
        # each preceded by its k_warp_prep (per-pair tables and tile bounds), whose bytes count too
        if "k_warp_prep" in r["Kernel_Name"] and int(r["Grid_Size"]) >= prep_threads:
            prep[r["Counter_Name"]].append(float(r["Counter_Value"]))
        if "k_warp_diff" not in r["Kernel_Name"]:
            continue
        if int(r["Grid_Size"]) < (w * h * b) // 64:
            continue
        vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
avg = lambda v: sum(v) / len(v) if v else 0.0  # noqa: E731
fetch_kib = avg(vals["FETCH_SIZE"]) + avg(prep["FETCH_SIZE"])
write_kib = avg(vals["WRITE_SIZE"]) + avg(prep["WRITE_SIZE"])
read_b = 2.0 * fetch_kib * 1024
write_b = write_kib * 1024
res = dict(kernel="k_warp_prep + k_warp_diff", config=config, launches=len(vals["FETCH_SIZE"]),
           prep_launches=len(prep["FETCH_SIZE"]),
           fetch_size_kib=round(fetch_kib, 1), write_size_kib=round(write_kib, 1),
           read_bytes_per_launch=int(read_b), write_bytes_per_launch=int(write_b),
           hbm_bytes_per_launch=int(read_b + write_b), algorithmic_bytes_per_launch=3 * w * h * b,
           correction="read = 2 x FETCH_SIZE (gfx950), write = WRITE_SIZE",
           source=os.path.basename(os.path.normpath(d)), src_sha256=bench_stamp(d))
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
