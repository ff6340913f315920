"""Dump per-(level, point) LK iteration counts of the 1080p synthetic pair (MDX_LK_DEBUG=1).

Run on the GPU box: MDX_LK_DEBUG=1 python scripts/lk_iters.py -> gpurun_out/lk_iters.npz
"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import motion_detection_amd as m

out = {}
for (w, h, ps, seed) in [(1920, 1080, 10, 1), (1920, 1080, 10, 2), (640, 480, 3, 7)]:
    a, b, _ = m.synth_pair(seed, w, h, 1)
    with m.Context(0, w, h, 1, pixel_step=ps) as c:
        r = c.flow_warp_diff(a, b)
        n = m.grid_count(w, h, ps)
        buf = np.zeros((8, n, 4), np.float32)
        rc = m.lib().mdx_debug_copy(c._h, 1, buf.ctypes.data_as(C.c_void_p), buf.nbytes)
        assert rc == 0, rc
        out[f"{w}x{h}_ps{ps}_s{seed}"] = buf
        print(w, h, ps, seed, "num_vectors", r.num_vectors)
np.savez_compressed("gpurun_out/lk_iters.npz", **out)
