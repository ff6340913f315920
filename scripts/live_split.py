import time, numpy as np, sys, json
sys.path.insert(0, '.')
import motion_detection_amd as mdx
w, h = 1920, 1080
a, b, _ = mdx.synth_pair(20141110, w, h, 3, 16)
ctx = mdx.Context(0, w, h, 4, pixel_step=10, min_vector_size=1.0)
for k in range(5):
    ctx.ring_push(a if k % 2 == 0 else b, 5)
ctx.ring_trajectory(w, h, 5)
tp, tt = [], []
for k in range(20):
    t0 = time.perf_counter(); ctx.ring_push(b if k % 2 == 0 else a, 5); ctx.sync(); t1 = time.perf_counter()
    ctx.ring_trajectory(w, h, 5); t2 = time.perf_counter()
    tp.append(t1 - t0); tt.append(t2 - t1)
print(json.dumps(dict(push_ms=round(1e3 * np.median(tp), 3), traj_ms=round(1e3 * np.median(tt), 3))))
