import ctypes as C, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import motion_detection_amd as m
w, h, ps, seed = 640, 480, 3, 7
a, b, _ = m.synth_pair(seed, w, h, 1)
out = {}
with m.Context(0, w, h, 1, pixel_step=ps) as c:
    r = c.flow_warp_diff(a, b)
    L = m.lib()
    for which, nm, nbytes in [(2, "pyr1", 4 << 20), (3, "pyr2", 4 << 20), (4, "der", 8 << 20), (5, "cls", 64 << 20)]:
        buf = np.zeros(nbytes, np.uint8)
        rc = L.mdx_debug_copy(c._h, which, buf.ctypes.data_as(C.c_void_p), buf.nbytes)
        out[nm] = buf if rc == 0 else np.zeros(1, np.uint8)
        print(nm, rc)
np.savez_compressed("gpurun_out/lk_dbg2.npz", **out)
