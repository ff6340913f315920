"""One row band of an 8K RGB pair (config C4: the share of one GPU when the frame is split over
8), on one context, F = 1: wall time per band call (flow + fit/warp, host-synchronised), for
rocprofv3 kernel traces of a band (GPU box).
Usage: python scripts/c4_band.py [band 0..7] [reps]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import motion_detection_amd as mdx
from motion_detection_amd import rowtile


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    w, h, K = 7680, 4320, 8
    a, b, _ = mdx.synth_pair(20141105 + 4, w, h, 3, 16)
    c = mdx.Context(0, w, h, 1, pixel_step=10, min_vector_size=1.0)
    n = mdx.grid_count(w, h, 10)
    d = {q: c.dev_alloc(sz) for q, sz in dict(i1=a.nbytes, i2=b.nbytes, np=n * 8, st=n, cand=96, cands=K * 96,
                                              mask=w * h, num=4).items()}
    c.h2d(d["i1"], a)
    c.h2d(d["i2"], b)
    y0, y1 = rowtile.band_rows(h, K, k)
    for it in range(reps + 2):
        if it == 2:
            c.device_sync()
            t0 = time.perf_counter()
        c.band_flow_dev(d["i1"], d["i2"], w, h, w * 3, mdx.FMT_RGB8, y0, y1, d["np"], d["st"], d["cand"])
        c.band_fit_warp_dev(1, d["cand"], y0, y1, d["mask"] + y0 * w, 0, d["num"])
    c.device_sync()
    print(f"band {k} of {K} rows [{y0}, {y1}): {(time.perf_counter() - t0) / reps * 1e3:.3f} ms per band (F = 1)")
    for p in d.values():
        c.dev_free(p)
    c.close()


if __name__ == "__main__":
    main()
