"""GPU box debug aid for k_warp_diff: with a WX_DEBUG_VAL build (MDX_LIB_PATH=.../libmdx_dbg.so)
the 'mask' holds the warped values; compare them with the oracle's warpPerspective."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import motion_detection_amd as mdx
from oracle import pyoracle as oracle

w, h = 640, 480
a, b, Ht = mdx.synth_pair(500, w, h, 1)
ctx = mdx.Context(0, w, h, 1)
d1, d2, dH, dM = (ctx.dev_alloc(x) for x in (a.nbytes, b.nbytes, 72, w * h))
ctx.h2d(d1, a); ctx.h2d(d2, b); ctx.h2d(dH, np.ascontiguousarray(Ht, dtype=np.float64))
ctx.warp_diff_dev(1, d1, d2, w, h, w, w * h, dH, dM); ctx.sync()
out = np.empty((h, w), np.uint8); ctx.d2h(out, dM)
M = oracle.invert3x3(Ht)
warped = oracle.warp_perspective(a, M)
bad = np.argwhere(out != warped)
print("M", M.tolist())
print(f"{len(bad)} warped values differ")
for y, x in bad[:20]:
    X0 = M[0, 0] * (x & ~63) + M[0, 1] * y + M[0, 2]; Y0 = M[1, 0] * (x & ~63) + M[1, 1] * y + M[1, 2]
    X = int(np.rint((X0 + M[0, 0] * (x & 63)) * 32)); Y = int(np.rint((Y0 + M[1, 0] * (x & 63)) * 32))
    sx, sy = X >> 5, Y >> 5
    taps = [int(a[sy + i, sx + j]) if 0 <= sy + i < h and 0 <= sx + j < w else 0 for i in (0, 1) for j in (0, 1)]
    print(f"  ({y},{x}) gpu {out[y, x]} ref {warped[y, x]}  X {X} Y {Y} fx {X & 31} fy {Y & 31} taps {taps}")
if len(bad):
    diff = out.astype(int) - warped.astype(int)
    print("diff values:", np.unique(diff[out != warped])[:30])
    print("x mod 4:", np.bincount(bad[:, 1] % 4), " x mod 128 hist nonzero:", np.nonzero(np.bincount(bad[:, 1] % 128))[0][:30])
