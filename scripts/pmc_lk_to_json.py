"""Per-step LK counters from scripts/pmc_lk.sh's passes.
Usage: python scripts/pmc_lk_to_json.py <dir> [steps covered by the run | auto]
auto (default): the steps are counted as the 1080p x 32 k_warp_diff launches (one per step; the bench
also runs its value_unpipelined steps under the profiler)."""
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

def fallbacks(d):
    """lk_fallbacks of every profiled bench line (one per pass)."""
    out = []
    for f in sorted(glob.glob(os.path.join(d, "p*.json"))):
        for line in open(f):
            line = line.strip()
            if line.startswith("{"):
                try:
                    out.append(json.loads(line).get("lk_fallbacks"))
                except ValueError:
                    pass
    return out


d = sys.argv[1]
steps_arg = sys.argv[2] if len(sys.argv) > 2 else "auto"
tot = defaultdict(float)
per_kernel = defaultdict(lambda: defaultdict(float))
warp_ids = defaultdict(set)
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "k_warp_diff" in k and int(r["Grid_Size"]) >= 1920 * 1080 * 32 // 64:
            warp_ids[f].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
        if "k_lk" not in k:
            continue
        name = k.split("(")[0].split("<")[0].replace("void ", "").replace("mdx::", "")
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        per_kernel[name][r["Counter_Name"]] += float(r["Counter_Value"])
# counters come from several passes, each over the same run: steps = launches seen per pass
steps = int(steps_arg) if steps_arg != "auto" else max(len(v) for v in warp_ids.values())
bench = json.load(open(f"{d}/p1.json"))
cfg = bench["config"]
w, h = (int(x) for x in cfg["frame"].split("x"))
out = {"kernels": "k_lk_class + k_lk_A + k_lk_iter", "config": f"{w}x{h}x{cfg['batch_per_gpu']}_ps{cfg['pixel_step']}",
       "steps_counted": steps, "sq_insts_valu_per_step": tot["SQ_INSTS_VALU"] / steps,
       "sq_insts_lds_per_step": tot["SQ_INSTS_LDS"] / steps,
       "per_kernel_valu_per_step": {k: v["SQ_INSTS_VALU"] / steps for k, v in per_kernel.items()},
       "counters_per_step": {k: v / steps for k, v in sorted(tot.items())},
       "source": "scripts/pmc_lk.sh (rocprofv3 --pmc, two passes, level dataflow ON: where counter collection "
                 "serializes kernels the waits give up and the levels are recomputed in sequence inside each call "
                 "(lk_fallbacks below, from the profiled bench line))",
       "lk_fallbacks": fallbacks(d),
       "src_sha256": bench_stamp(d)}
print(json.dumps(out, indent=1))
