"""Per-step LK counters from scripts/pmc_lk.sh's passes.
Usage: python scripts/pmc_lk_to_json.py <dir> <steps covered by the run (warmup + timed)>"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


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

d, steps = sys.argv[1], int(sys.argv[2])
tot = defaultdict(float)
per_kernel = defaultdict(lambda: defaultdict(float))
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "k_lk" not in k:
            continue
        name = k.split("(")[0].split("<")[0].replace("void ", "").replace("mdx::", "")
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        per_kernel[name][r["Counter_Name"]] += float(r["Counter_Value"])
bench = json.load(open(f"{d}/p1.json"))
cfg = bench["config"]
w, h = (int(x) for x in cfg["frame"].split("x"))
out = {"kernels": "k_lk_class + k_lk_A + k_lk_iter", "config": f"{w}x{h}x{cfg['batch_per_gpu']}_ps{cfg['pixel_step']}",
       "steps_counted": steps, "sq_insts_valu_per_step": tot["SQ_INSTS_VALU"] / steps,
       "sq_insts_lds_per_step": tot["SQ_INSTS_LDS"] / steps,
       "per_kernel_valu_per_step": {k: v["SQ_INSTS_VALU"] / steps for k, v in per_kernel.items()},
       "counters_per_step": {k: v / steps for k, v in sorted(tot.items())},
       "source": "scripts/pmc_lk.sh (rocprofv3 --pmc, two passes)", "src_sha256": bench_stamp(d)}
print(json.dumps(out, indent=1))
