"""Compare LK v1 (single kernel) and v2 (class planes) against the oracle; print diffs."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import motion_detection_amd as m
from oracle import pyoracle as po

def run(impl, a, b, ps):
    os.environ["MDX_LK_IMPL"] = str(impl)
    h, w = a.shape
    with m.Context(0, w, h, 1, pixel_step=ps) as c:
        return c.flow_warp_diff(a, b)

for (w, h, ps, seed) in [(640, 480, 3, 7), (1920, 1080, 10, 20141106)]:
    a, b, _ = m.synth_pair(seed, w, h, 1)
    r1, r2 = run(1, a, b, ps), run(2, a, b, ps)
    ref = po.calculate_optical_flow(a, b, nthreads=8, pixel_step=ps)
    ny = (h + ps - 1) // ps
    d = np.nonzero((r2.next_pts.view(np.uint32) != ref["next_pts"].view(np.uint32)).any(1) | (r2.status != ref["status"]))[0]
    d1 = np.nonzero((r1.next_pts.view(np.uint32) != ref["next_pts"].view(np.uint32)).any(1))[0]
    print(f"{w}x{h} ps{ps}: v1 diffs {len(d1)}, v2 diffs {len(d)}")
    for i in d[:10]:
        print(f"  pt {i} grid ({(i//ny)*ps},{(i%ny)*ps}) v2 {r2.next_pts[i]} st{r2.status[i]}  ref {ref['next_pts'][i]} st{ref['status'][i]}")
