"""Per-level LK work of the bench workload: iterations per point and the group lockstep.

Runs the bench's 1080p x 32 step (4 distinct synthetic pairs) with MDX_LK_DEBUG=1 and reads the
per-(pair, level, point) trace k_lk_iter writes (npx, npy, iterations, status).  Per level it prints
the tracked points, the Newton iterations they execute, and what the persistent slots execute:
a group of G class members iterates max(its points) times, so the slot cost is G x that sum.  The
grouping is the host plan's (mdx_api.cpp ensure_class_plan: one residue class's members along a
grid row, in x order, padded to G); both G = 4 and G = 8 are evaluated per level.

With --times <kernel_trace.csv> (a rocprofv3 --kernel-trace of the bench with MDX_LK_FLOW=0, so
the levels run in sequence) it joins the mean k_lk_iter duration per level and prints ns per
point-iteration and per slot-iteration.
Usage (GPU box): MDX_LK_DEBUG=1 python scripts/lk_level_diag.py [--times run_kernel_trace.csv]
"""
import argparse
import csv
import ctypes as C
import math
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import motion_detection_amd as m

UW4 = [48, 56, 64, 72, 80, 96, 128]
UW8 = [80, 112, 128, 256, 512]


def fl32(x):
    return float(np.float32(x))


def ipx_of(gx, ps, level):
    return int(math.floor(fl32(fl32(gx * ps) * fl32(1.0 / (1 << level)) - 19.5)))


def groups(nx, ps, level, G):
    """Column groups of one grid row: lists of gx (host plan order), and the union width."""
    msk = (1 << level) - 1
    runs = defaultdict(list)
    for i in range(nx):
        runs[(i * ps) & msk].append(i)
    out, u = [], 0
    for r in runs.values():
        for q in range(0, len(r), G):
            g = r[q:q + G]
            out.append(g)
            u = max(u, ipx_of(g[-1], ps, level) - ipx_of(g[0], ps, level) + 40)
    return out, u


def plan_g(nx, ps, level):
    _, u4 = groups(nx, ps, level, 4)
    _, u8 = groups(nx, ps, level, 8)
    uw4 = next((x for x in UW4 if x >= u4), 0)
    uw8 = next((x for x in UW8 if x >= u8), 0)
    pieces = lambda s, uw: (s * uw * 8 + 1023) // 1024
    g4 = uw4 > 0 and (uw8 == 0 or pieces(4, uw4) <= pieces(2, uw8))
    return (4, uw4) if g4 else (8, uw8)


def level_times(path):
    """Mean duration (us) of each level's k_lk_iter launch (dispatch order maxL..0 within a step)."""
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    per = defaultdict(list)
    n = None
    for r in rows:
        name = (r.get("Kernel_Name") or r.get("Name") or "")
        if "k_front" in name and n is not None and n > 0:
            n = 0
        if "k_lk_iter" in name:
            if n is None:
                n = 0
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            per[n].append(dur)
            n += 1
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--times", default=None)
    ap.add_argument("--w", type=int, default=1920)
    ap.add_argument("--h", type=int, default=1080)
    ap.add_argument("--ps", type=int, default=10)
    args = ap.parse_args()
    assert os.environ.get("MDX_LK_DEBUG") == "1", "run with MDX_LK_DEBUG=1"
    w, h, ps, B = args.w, args.h, args.ps, 32
    uniq = [m.synth_pair(20141105 + i, w, h, 1) for i in range(4)]
    g1 = np.stack([uniq[i % 4][0] for i in range(B)])
    g2 = np.stack([uniq[i % 4][1] for i in range(B)])
    nx, ny = (w + ps - 1) // ps, (h + ps - 1) // ps
    n = nx * ny
    with m.Context(0, w, h, B, pixel_step=ps, min_vector_size=1.0) as c:
        b1, b2 = c.dev_alloc(g1.nbytes), c.dev_alloc(g2.nbytes)
        c.h2d(b1, g1)
        c.h2d(b2, g2)
        c.flow_warp_diff_batch_dev(B, b1, b2, w, h, w, w * h, m.FMT_GRAY8)
        c.sync()
        nlev = 5
        buf = np.zeros((B, 8, n, 4), np.float32)
        rc = m.lib().mdx_debug_copy(c._h, 1, buf.ctypes.data_as(C.c_void_p), B * nlev * n * 16)
        assert rc == 0, rc
        c.dev_free(b1)
        c.dev_free(b2)
    it = buf[:4, :nlev, :, 2].astype(np.int64)          # the 4 distinct pairs
    times = level_times(args.times) if args.times else {}
    tot = defaultdict(float)
    print(f"{w}x{h} ps {ps}: {n} grid points per pair; per level over the 4 distinct pairs (x8 in the step)")
    for L in range(nlev - 1, -1, -1):
        G, UW = plan_g(nx, ps, L)
        line = [f"level {L}: plan G={G} UW={UW}"]
        pit = int(it[:, L].sum())
        tracked = int((it[:, L] > 0).sum())
        line.append(f"tracked {tracked / 4:.0f}/pair, iters {pit / 4:.0f}/pair ({pit / max(tracked, 1):.2f}/tracked pt)")
        for g in (4, 8):
            gl, _ = groups(nx, ps, L, g)
            cost = 0
            for p in range(4):
                itp = it[p, L].reshape(nx, ny)       # point k = gx * ny + gy
                for members in gl:
                    mx = itp[members, :].max(axis=0)  # per grid row
                    cost += int(mx.sum()) * g
            line.append(f"G={g}: slot-iters/point-iters {cost / max(pit, 1):.3f}")
            if g == G:
                tot["slot"] += cost
                slot_cost = cost
        tot["pit"] += pit
        print("  " + "; ".join(line))
        k = nlev - 1 - L
        if k in times:
            us = float(np.mean(times[k]))
            print(f"    k_lk_iter {us:.1f} us mean over {len(times[k])} launches: "
                  f"{us * 1e3 / (pit * 8):.4f} ns per point-iteration, "
                  f"{us * 1e3 / (slot_cost * 8):.4f} ns per slot point-iteration (step = 8x the 4 pairs)")
    print(f"all levels: point-iterations {tot['pit'] * 8:.0f} per step, slot/point {tot['slot'] / tot['pit']:.3f}")


if __name__ == "__main__":
    main()
