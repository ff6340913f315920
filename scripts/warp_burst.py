"""A burst of k_warp_diff launches after idle (the roofline leg's workload: 4K gray x 32 pairs, the
generator's affine true H), for the per-launch clock diagnosis of the warp's burst transient.

Usage (GPU box):
  python scripts/warp_burst.py [launches] [idle_s] [--probe]
run under `rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES ...` (per-dispatch cycles and
durations: scripts/warp_burst.sh) or with a stamped diagnostic library (MDX_LIB_PATH, built with
-DMDX_WARP_STAMP=1: in-kernel s_memtime / s_memrealtime per sampled workgroup, read back here).
--probe launches the copy probe k_stream3 instead (the same buffers).
"""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import motion_detection_amd as mdx

STAMP_WHICH = 99          # mdx_debug_copy selector of the diagnostic build's stamp table
STAMP_LAUNCHES = 1024     # its ring of launches
STAMP_SAMPLES = 64        # sampled workgroups per launch


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    n = int(args[0]) if args else 300
    idle = float(args[1]) if len(args) > 1 else 2.0
    probe = "--probe" in sys.argv
    w, h, B = 3840, 2160, 32
    a, b, Ht = mdx.synth_pair(20141105 + 77, w, h, 1, 16)
    g1 = np.ascontiguousarray(np.broadcast_to(a, (B, h, w)))
    g2 = np.ascontiguousarray(np.broadcast_to(b, (B, h, w)))
    Hb = np.ascontiguousarray(np.broadcast_to(np.asarray(Ht, np.float64).reshape(3, 3), (B, 3, 3)))
    c = mdx.Context(0, 64, 64, 1)
    e1, e2, eH, eM = c.dev_alloc(g1.nbytes), c.dev_alloc(g2.nbytes), c.dev_alloc(Hb.nbytes), c.dev_alloc(B * w * h)
    c.h2d(e1, g1)
    c.h2d(e2, g2)
    c.h2d(eH, Hb)
    c.warp_diff_dev(B, e1, e2, w, h, w, w * h, eH, eM)
    c.device_sync()
    time.sleep(idle)
    t0 = time.perf_counter()
    for _ in range(n):
        if probe:
            c.probe_stream3_dev(B * w * h, e1, e2, eM)
        else:
            c.warp_diff_dev(B, e1, e2, w, h, w, w * h, eH, eM)
    c.device_sync()
    el = time.perf_counter() - t0
    out = {"launches": n, "idle_s": idle, "kernel": "k_stream3" if probe else "k_warp_diff",
           "wall_us_per_launch": round(el / n * 1e6, 2)}
    if os.environ.get("MDX_LIB_PATH") and not probe:
        st = np.zeros((STAMP_LAUNCHES, STAMP_SAMPLES, 4), np.uint64)
        rc = mdx.lib().mdx_debug_copy(c._h, STAMP_WHICH, st.ctypes.data_as(C.c_void_p), st.nbytes)
        if rc == 0:
            # launch 1 is the one before the idle; the burst is launches 2 .. n + 1
            rows = []
            for i in range(2, min(n + 2, STAMP_LAUNCHES)):
                s = st[i]
                ok = s[:, 3] > s[:, 1]
                if not ok.any():
                    continue
                dt_clk = (s[ok, 2].astype(np.int64) - s[ok, 0].astype(np.int64))
                dt_ref = (s[ok, 3].astype(np.int64) - s[ok, 1].astype(np.int64))
                mhz = np.median(dt_clk / np.maximum(dt_ref, 1)) * 100.0
                span_us = (s[ok, 3].max() - s[ok, 1].min()) / 100.0
                rows.append((i, round(float(mhz), 1), round(float(np.median(dt_clk)), 0), round(float(span_us), 1)))
            out["stamps"] = {"columns": "launch, in-kernel MHz (median over sampled workgroups), median workgroup "
                                        "cycles, launch span us (first start .. last end of the sampled workgroups)",
                             "rows": rows}
    print(json.dumps(out))
    for p in (e1, e2, eH, eM):
        c.dev_free(p)
    c.close()


if __name__ == "__main__":
    main()
