"""HBM traffic of one whole default-bench step (1080p x 32 pairs), per kernel and in total, from a
scripts/pmc_sets.sh run with a FETCH_SIZE pass and a WRITE_SIZE pass over
`bench.py --steps 2 --warmup 1 --no-cpu --no-roofline --no-live --no-4k --no-lk-roofline`.

gfx950 correction (MI355X_MICROARCH.md, HBM section): read bytes = 2 x FETCH_SIZE KiB; WRITE_SIZE
is exact.  Steps are counted by the k_warp_diff launches of the 1080p batch (one per step).
Compared with SURVEY §8d's algorithmic 9 B/px (pyramids of both frames, one LK sweep over both,
warp + diff) and with the class planes' own bytes.
Usage: python scripts/pmc_step_to_json.py gpurun_out/pmc_<tag> [out.json]
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

d = sys.argv[1]
out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(__file__), "..", "profiles", "pmc_step.json")
W, H, B = 1920, 1080, 32
per = collections.defaultdict(lambda: collections.defaultdict(float))
steps = 0
for f in sorted(glob.glob(os.path.join(d, "*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        per[name][r["Counter_Name"]] += float(r["Counter_Value"])
        if r["Counter_Name"] == "WRITE_SIZE" and "k_warp_diff" in name and int(r["Grid_Size"]) >= W * H * B // 64:
            steps += 1
if steps == 0:
    sys.exit("no 1080p k_warp_diff launches found")
rows = []
tot_r = tot_w = 0.0
for name, c in per.items():
    rb = 2.0 * c.get("FETCH_SIZE", 0.0) * 1024 / steps
    wb = c.get("WRITE_SIZE", 0.0) * 1024 / steps
    tot_r += rb
    tot_w += wb
    rows.append(dict(kernel=name, read_mb=round(rb / 1e6, 1), write_mb=round(wb / 1e6, 1)))
rows.sort(key=lambda x: -(x["read_mb"] + x["write_mb"]))
px = W * H * B
res = dict(workload=f"{W}x{H} gray, {B} pairs per step, pixel_step 10 (bench.py default step)", steps=steps,
           config=f"{W}x{H}x{B}_ps10", src_sha256=bench_stamp(d),
           hbm_read_mb_per_step=round(tot_r / 1e6, 1), hbm_write_mb_per_step=round(tot_w / 1e6, 1),
           hbm_bytes_per_px=round((tot_r + tot_w) / px, 2), algorithmic_bytes_per_px=9.0,
           per_kernel=rows, correction="read = 2 x FETCH_SIZE (gfx950), write = WRITE_SIZE",
           source=os.path.basename(os.path.normpath(d)),
           note="level dataflow ON (round 5): where counter collection serializes kernels, the LK waits give up "
                "and the levels are recomputed in sequence inside each call (see the bench lines' lk_fallbacks)")
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "per_kernel"}))
for r in rows[:15]:
    print(r)
