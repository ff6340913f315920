"""Would pass 0 of the live chain (grid start points) be faster through the class-plane LK?

Times, on one 1080p rgb8 pair: (a) the class-plane LK (k_lk_class*, k_lk_A_rows, k_lk_iter) of the
pair path at batch 1 -- the LK stage of mdx_flow_warp_diff_batch_dev by HIP events; (b) one
trajectory pass through the point LK (a ring of 2 frames: mdx_ring_trajectory, one k_lk pass), and
(c) the node's 5-frame ring callback, both by wall clock.  Run on the GPU box, ideally under
`rocprofv3 --kernel-trace --stats` for the per-kernel split.
Usage: python scripts/pass0_lk.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import motion_detection_amd as m


def main():
    w, h, reps = 1920, 1080, 20
    a, b, _ = m.synth_pair(20141110, w, h, 3, 16)
    out = {}
    with m.Context(0, w, h, 1, pixel_step=10, min_vector_size=1.0) as c:
        n = m.grid_count(w, h, 10)
        d1, d2 = c.dev_alloc(a.nbytes), c.dev_alloc(b.nbytes)
        o = {k: c.dev_alloc(sz) for k, sz in dict(np=n * 8, st=n, mask=w * h, H=72, num=4).items()}
        c.h2d(d1, a); c.h2d(d2, b)
        call = lambda: c.flow_warp_diff_batch_dev(1, d1, d2, w, h, 3 * w, 3 * w * h, m.FMT_RGB8,  # noqa: E731
                                                  d_next_pts=o["np"], d_status=o["st"], d_mask=o["mask"],
                                                  d_H=o["H"], d_num_vectors=o["num"])
        for _ in range(3):
            call()
        c.sync()
        c.enable_timing(True)
        for _ in range(reps):
            call()
        c.sync()
        st = c.stage_ms()
        out["class_plane_lk_ms"] = round(st["lk"] / st["calls"], 3)
        out["pair_path_total_ms"] = round(st["total"] / st["calls"], 3)
        for p in [d1, d2] + list(o.values()):
            c.dev_free(p)
        for nimg in (2, 5):
            c.ring_reset()
            frames = [a if k % 2 == 0 else b for k in range(nimg + 8)]
            for f in frames[:nimg]:
                c.ring_push(f, nimg)
            res = c.ring_trajectory(w, h, nimg)
            ts = []
            for f in frames[nimg:]:
                t0 = time.perf_counter()
                c.ring_push(f, nimg)
                res = c.ring_trajectory(w, h, nimg, out=res)
                ts.append(time.perf_counter() - t0)
            out[f"ring_callback_{nimg}_frames_ms"] = round(float(np.median(ts)) * 1e3, 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
