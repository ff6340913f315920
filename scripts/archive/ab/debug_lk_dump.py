"""Dump LK v2 internals (A sums, per-level trace) for offline comparison with the oracle."""
import ctypes as C, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["MDX_LK_DEBUG"] = "1"
os.environ["MDX_LK_DEBUG_PT"] = "4394"
import numpy as np
import motion_detection_amd as m
w, h, ps, seed = 640, 480, 3, 7
a, b, _ = m.synth_pair(seed, w, h, 1)
with m.Context(0, w, h, 1, pixel_step=ps) as c:
    r = c.flow_warp_diff(a, b)
    n = m.grid_count(w, h, ps); nlev = 4
    A = np.zeros((nlev, n, 4), np.float32); T = np.zeros((nlev * n + 8 * 64, 4), np.float32)
    assert m.lib().mdx_debug_copy(c._h, 0, A.ctypes.data_as(C.c_void_p), A.nbytes) == 0
    assert m.lib().mdx_debug_copy(c._h, 1, T.ctypes.data_as(C.c_void_p), T.nbytes) == 0
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/lk_dbg.npz", A=A, T=T[:nlev * n].reshape(nlev, n, 4), IT=T[nlev * n:].reshape(8, 16, 4, 4), next_pts=r.next_pts, status=r.status)
print("dumped", A.shape)
