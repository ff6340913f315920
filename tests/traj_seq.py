"""Synthetic frame sequences for the trajectory tests (test helper, not a test module).

A textured base frame (mdx_synth_pair's frame 1) seen through a camera that moves by a fixed
similarity per frame (small rotation + scale + translation), plus one patch that moves on its own
and +-2 LSB noise; frame k samples the base at M^k (the oracle's warpPerspective restatement).
"""
import numpy as np


def camera_step(w, h, tx=2.3, ty=-1.4, deg=0.3, s=1.004):
    c, si = np.cos(np.radians(deg)) * s, np.sin(np.radians(deg)) * s
    cx, cy = w / 2, h / 2
    return np.array([[c, -si, cx - c * cx + si * cy + tx], [si, c, cy - si * cx - c * cy + ty], [0, 0, 1.0]])


def sequence(mdx, oracle, w, h, n, seed=7, channels=1, step=None, patch=True):
    base, _, _ = mdx.synth_pair(seed, w, h, 1)
    rng = np.random.default_rng(seed)
    M = camera_step(w, h) if step is None else step
    frames = []
    Mk = np.eye(3)
    for k in range(n):
        f = oracle.warp_perspective(base, np.linalg.inv(Mk)) if k else base.copy()
        if patch:
            pw, ph = w // 5, h // 5
            x0, y0 = w // 3 + 5 * k, h // 3 + 3 * k
            f[y0:y0 + ph, x0:x0 + pw] = base[h // 2:h // 2 + ph, w // 2:w // 2 + pw][:f[y0:y0 + ph, x0:x0 + pw].shape[0],
                                                                                   :f[y0:y0 + ph, x0:x0 + pw].shape[1]]
        noise = rng.integers(-2, 3, f.shape)
        f = np.clip(f.astype(np.int16) + noise, 0, 255).astype(np.uint8)
        if channels == 3:
            f = np.repeat(f[:, :, None], 3, axis=2)
            f[:, :, 0] = np.clip(f[:, :, 0].astype(np.int16) + rng.integers(-3, 4, (h, w)), 0, 255)
        frames.append(np.ascontiguousarray(f))
        Mk = M @ Mk
    return frames
