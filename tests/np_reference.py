"""Independent numpy restatement of the reference hot path (test infrastructure).

A second, separately written restatement of the OpenCV 2.4.8 semantics that
OpticalFlowCalculator::calculateOpticalFlow (reference
common/src/optical_flow_calculator.cpp:30-130) calls.  It exists only to pin the C
oracle (oracle/mdx_oracle.c): the two are written independently (scalar C loops vs.
numpy vectorised over points / pixels) and must agree bit for bit.  It never ships to the
GPU box path and nothing in the product imports it.
"""
from __future__ import annotations

import math
import struct

import numpy as np


def reflect101(p: np.ndarray | int, n: int):
    """borderInterpolate(p, n, BORDER_REFLECT_101), vectorised (any number of folds)."""
    p = np.asarray(p, dtype=np.int64)
    if n == 1:
        return np.zeros_like(p)
    period = 2 * n - 2
    q = np.mod(p, period)
    return np.where(q < n, q, period - q)


def to_gray(img: np.ndarray) -> np.ndarray:
    """cvtColor(CV_BGR2GRAY) applied to rgb8 data (node.cpp:271 then :50)."""
    if img.ndim == 2:
        return img.copy()
    s = img.astype(np.int64)
    return ((s[..., 0] * 1868 + s[..., 1] * 9617 + s[..., 2] * 4899 + 8192) >> 14).astype(np.uint8)


def pyrdown(src: np.ndarray) -> np.ndarray:
    h, w = src.shape
    dh, dw = (h + 1) // 2, (w + 1) // 2
    k = np.array([1, 4, 6, 4, 1], dtype=np.int64)
    s = src.astype(np.int64)
    xs = reflect101(2 * np.arange(dw)[:, None] + np.arange(5)[None, :] - 2, w)
    ys = reflect101(2 * np.arange(dh)[:, None] + np.arange(5)[None, :] - 2, h)
    hor = (s[:, xs] * k[None, None, :]).sum(-1)          # h x dw
    ver = (hor[ys, :] * k[None, :, None]).sum(1)          # dh x dw
    return ((ver + 128) >> 8).astype(np.uint8)


def scharr(src: np.ndarray) -> np.ndarray:
    """Returns int16 (h, w, 2) = (Ix, Iy); borders reflect-101 (calcSharrDeriv)."""
    h, w = src.shape
    s = src.astype(np.int64)
    ym = reflect101(np.arange(h) - 1, h)
    yp = reflect101(np.arange(h) + 1, h)
    t0 = (s[ym] + s[yp]) * 3 + s * 10
    t1 = s[yp] - s[ym]
    xm = reflect101(np.arange(w) - 1, w)
    xp = reflect101(np.arange(w) + 1, w)
    ix = t0[:, xp] - t0[:, xm]
    iy = (t1[:, xm] + t1[:, xp]) * 3 + t1 * 10
    return np.stack([ix, iy], -1).astype(np.int16)


def build_pyramid(gray: np.ndarray, win: int, max_level: int):
    """Unpadded levels + level count (buildOpticalFlowPyramid stop rule)."""
    levels = [gray]
    h, w = gray.shape
    for lvl in range(max_level + 1):
        if lvl > 0:
            levels.append(pyrdown(levels[-1]))
        w2, h2 = (w + 1) // 2, (h + 1) // 2
        if w2 <= win or h2 <= win:
            return levels, lvl
        w, h = w2, h2
    return levels, max_level


def pad_reflect(img: np.ndarray, pad: int) -> np.ndarray:
    h, w = img.shape
    ys = reflect101(np.arange(-pad, h + pad), h)
    xs = reflect101(np.arange(-pad, w + pad), w)
    return img[ys][:, xs]


def pad_zero(d: np.ndarray, pad: int) -> np.ndarray:
    return np.pad(d, ((pad, pad), (pad, pad), (0, 0)))


def _round_half_even_f32(v: np.ndarray) -> np.ndarray:
    return np.rint(v.astype(np.float32)).astype(np.int64)


def _weights(a: np.ndarray, b: np.ndarray):
    one = np.float32(1.0)
    s = np.float32(1 << 14)
    w00 = _round_half_even_f32(((one - a) * (one - b)).astype(np.float32) * s)
    w01 = _round_half_even_f32((a * (one - b)).astype(np.float32) * s)
    w10 = _round_half_even_f32(((one - a) * b).astype(np.float32) * s)
    w11 = (1 << 14) - w00 - w01 - w10
    return w00, w01, w10, w11


def lk(prev_levels, next_levels, max_level, pts, win=40, max_iters=10, eps=0.03, min_eig=1e-3):
    """calcOpticalFlowPyrLK with the SSE2 summation order, vectorised over points."""
    f32 = np.float32
    n = pts.shape[0]
    pad = win
    status = np.ones(n, dtype=bool)
    nextp = np.zeros((n, 2), dtype=np.float32)
    halfw = f32((win - 1) * 0.5)
    eps2 = eps * eps
    thr = f32(min_eig)
    yy, xx = np.meshgrid(np.arange(win), np.arange(win), indexing="ij")
    for level in range(max_level, -1, -1):
        I = pad_reflect(prev_levels[level], pad).astype(np.int64)
        Dv = pad_zero(scharr(prev_levels[level]), pad).astype(np.int64)
        J = pad_reflect(next_levels[level], pad).astype(np.int64)
        ih, iw = prev_levels[level].shape
        scale = f32(1.0 / (1 << level))
        pp = (pts * scale).astype(np.float32)
        if level == max_level:
            nextp = pp.copy()
        else:
            nextp = (nextp * f32(2.0)).astype(np.float32)
        pp = (pp - halfw).astype(np.float32)
        ip = np.floor(pp.astype(np.float64)).astype(np.int64)
        ok = (ip[:, 0] >= -win) & (ip[:, 0] < iw) & (ip[:, 1] >= -win) & (ip[:, 1] < ih)
        if level == 0:
            status &= ok
        idx = np.nonzero(ok)[0]
        if idx.size == 0:
            continue
        a = (pp[idx, 0] - ip[idx, 0].astype(np.float32)).astype(np.float32)
        b = (pp[idx, 1] - ip[idx, 1].astype(np.float32)).astype(np.float32)
        w00, w01, w10, w11 = _weights(a, b)
        oy = ip[idx, 1][:, None, None] + yy[None] + pad
        ox = ip[idx, 0][:, None, None] + xx[None] + pad
        w = [t[:, None, None] for t in (w00, w01, w10, w11)]
        Iw = (I[oy, ox] * w[0] + I[oy, ox + 1] * w[1] + I[oy + 1, ox] * w[2] + I[oy + 1, ox + 1] * w[3] + 256) >> 9
        Ix = (Dv[oy, ox, 0] * w[0] + Dv[oy, ox + 1, 0] * w[1] + Dv[oy + 1, ox, 0] * w[2] + Dv[oy + 1, ox + 1, 0] * w[3] + 8192) >> 14
        Iy = (Dv[oy, ox, 1] * w[0] + Dv[oy, ox + 1, 1] * w[1] + Dv[oy + 1, ox, 1] * w[2] + Dv[oy + 1, ox + 1, 1] * w[3] + 8192) >> 14
        # chain k = x mod 4, steps in (y, x) order: reshape (m, 40, 10, 4) -> (m, 4, 400)
        def chains(t):
            return t.reshape(t.shape[0], win, win // 4, 4).transpose(0, 3, 1, 2).reshape(t.shape[0], 4, -1)
        def seqsum(c):
            acc = np.zeros(c.shape[:2], dtype=np.float32)
            for s in range(c.shape[2]):
                acc = (acc + c[:, :, s]).astype(np.float32)
            return acc
        qa11 = seqsum(chains((Ix * Ix).astype(np.float32)))
        qa12 = seqsum(chains((Ix * Iy).astype(np.float32)))
        qa22 = seqsum(chains((Iy * Iy).astype(np.float32)))
        def comb_a(q):
            return (((q[:, 0] + q[:, 1]).astype(f32) + q[:, 2]).astype(f32) + q[:, 3]).astype(f32)
        fs = f32(1.0 / (1 << 20))
        A11 = (comb_a(qa11) * fs).astype(f32)
        A12 = (comb_a(qa12) * fs).astype(f32)
        A22 = (comb_a(qa22) * fs).astype(f32)
        D = (A11 * A22 - A12 * A12).astype(f32)
        disc = ((A11 - A22) * (A11 - A22) + f32(4.0) * A12 * A12).astype(f32)
        mine = ((A22 + A11 - np.sqrt(disc)).astype(f32) / f32(2 * win * win)).astype(f32)
        good = ~((mine < thr) | (D < f32(np.finfo(np.float32).eps)))
        if level == 0:
            status[idx[~good]] = False
        for t, i in enumerate(idx):
            if not good[t]:
                continue
            Dinv = f32(f32(1.0) / D[t])
            nx, ny = f32(nextp[i, 0] - halfw), f32(nextp[i, 1] - halfw)
            pdx = pdy = f32(0.0)
            for j in range(max_iters):
                inx, iny = int(math.floor(float(nx))), int(math.floor(float(ny)))
                jh, jw = next_levels[level].shape
                if inx < -win or inx >= jw or iny < -win or iny >= jh:
                    if level == 0:
                        status[i] = False
                    break
                aa = np.array([f32(nx - f32(inx))], dtype=f32)
                bb = np.array([f32(ny - f32(iny))], dtype=f32)
                v00, v01, v10, v11 = (int(q[0]) for q in _weights(aa, bb))
                jy = iny + yy + pad
                jx = inx + xx + pad
                Jw = (J[jy, jx] * v00 + J[jy, jx + 1] * v01 + J[jy + 1, jx] * v10 + J[jy + 1, jx + 1] * v11 + 256) >> 9
                diff = Jw - Iw[t]
                c1 = chains((diff * Ix[t])[None].astype(np.float32))[0]
                c2 = chains((diff * Iy[t])[None].astype(np.float32))[0]
                q1 = seqsum(c1[None])[0]
                q2 = seqsum(c2[None])[0]
                b1 = f32(f32(q1[0] + q1[2]) + f32(q1[1] + q1[3]))
                b2 = f32(f32(q2[0] + q2[2]) + f32(q2[1] + q2[3]))
                b1 = f32(b1 * fs)
                b2 = f32(b2 * fs)
                dx = f32(f32(f32(A12[t] * b2) - f32(A22[t] * b1)) * Dinv)
                dy = f32(f32(f32(A12[t] * b1) - f32(A11[t] * b2)) * Dinv)
                nx = f32(nx + dx)
                ny = f32(ny + dy)
                nextp[i, 0] = f32(nx + halfw)
                nextp[i, 1] = f32(ny + halfw)
                if float(dx) * float(dx) + float(dy) * float(dy) <= eps2:
                    break
                if j > 0 and abs(float(f32(dx + pdx))) < 0.01 and abs(float(f32(dy + pdy))) < 0.01:
                    nextp[i, 0] = f32(nextp[i, 0] - f32(dx * f32(0.5)))
                    nextp[i, 1] = f32(nextp[i, 1] - f32(dy * f32(0.5)))
                    break
                pdx, pdy = dx, dy
        if level == 0:
            fp = (nextp - halfw).astype(np.float32)
            fi = np.floor(fp.astype(np.float64)).astype(np.int64)
            jh, jw = next_levels[0].shape
            oob = (fi[:, 0] < -win) | (fi[:, 0] >= jw) | (fi[:, 1] < -win) | (fi[:, 1] >= jh)
            status &= ~oob
    return nextp, status.astype(np.uint8)


# ------------------------------------------------------------------ perspective fit
def _hi(d):
    return struct.unpack("<Q", struct.pack("<d", d))[0] >> 32


def _lo(d):
    return struct.unpack("<Q", struct.pack("<d", d))[0] & 0xFFFFFFFF


def _sethi(d, hi):
    u = struct.unpack("<Q", struct.pack("<d", d))[0]
    return struct.unpack("<d", struct.pack("<Q", ((hi & 0xFFFFFFFF) << 32) | (u & 0xFFFFFFFF)))[0]


def fdlibm_hypot(x, y):
    ha = _hi(x) & 0x7FFFFFFF
    hb = _hi(y) & 0x7FFFFFFF
    if hb > ha:
        a, b, ha, hb = y, x, hb, ha
    else:
        a, b = x, y
    a = _sethi(a, ha)
    b = _sethi(b, hb)
    if ha - hb > 0x3C00000:
        return a + b
    k = 0
    if ha > 0x5F300000:
        if ha >= 0x7FF00000:
            return a + b
        ha -= 0x25800000; hb -= 0x25800000; k += 600
        a = _sethi(a, ha); b = _sethi(b, hb)
    if hb < 0x20B00000:
        if hb <= 0x000FFFFF:
            if (hb | _lo(b)) == 0:
                return a
            t1 = _sethi(0.0, 0x7FD00000)
            b *= t1; a *= t1; k -= 1022
        else:
            ha += 0x25800000; hb += 0x25800000; k -= 600
            a = _sethi(a, ha); b = _sethi(b, hb)
    w = a - b
    if w > b:
        t1 = _sethi(0.0, ha)
        t2 = a - t1
        w = math.sqrt(t1 * t1 - (b * (-b) - t2 * (a + t1)))
    else:
        a = a + a
        y1 = _sethi(0.0, hb)
        y2 = b - y1
        t1 = _sethi(0.0, ha + 0x00100000)
        t2 = a - t1
        w = math.sqrt(t1 * y1 - (w * (-w) - (t1 * y2 + t2 * b)))
    if k != 0:
        return _sethi(1.0, _hi(1.0) + (k << 20)) * w
    return w


def get_perspective_transform(src, dst):
    """getPerspectiveTransform -> solve(DECOMP_SVD): one-sided Jacobi on A's columns."""
    f32 = np.float32
    A = [[0.0] * 8 for _ in range(8)]
    bv = [0.0] * 8
    for i in range(4):
        sx, sy = f32(src[i][0]), f32(src[i][1])
        dx, dy = f32(dst[i][0]), f32(dst[i][1])
        A[i][0] = A[i + 4][3] = float(sx)
        A[i][1] = A[i + 4][4] = float(sy)
        A[i][2] = A[i + 4][5] = 1.0
        A[i][6] = float(f32(-sx * dx))
        A[i][7] = float(f32(-sy * dx))
        A[i + 4][6] = float(f32(-sx * dy))
        A[i + 4][7] = float(f32(-sy * dy))
        bv[i] = float(dx)
        bv[i + 4] = float(dy)
    m = n = 8
    At = [[A[k][i] for k in range(m)] for i in range(n)]
    Vt = [[1.0 if i == k else 0.0 for k in range(n)] for i in range(n)]
    W = [sum_seq([t * t for t in At[i]]) for i in range(n)]
    eps = np.finfo(np.float64).eps * 10
    for _ in range(max(m, 30)):
        changed = False
        for i in range(n - 1):
            for j in range(i + 1, n):
                a, b = W[i], W[j]
                p = sum_seq([At[i][k] * At[j][k] for k in range(m)])
                if abs(p) <= eps * math.sqrt(a * b):
                    continue
                p *= 2
                beta = a - b
                gamma = fdlibm_hypot(p, beta)
                if beta < 0:
                    delta = (gamma - beta) * 0.5
                    s = math.sqrt(delta / gamma)
                    c = p / (gamma * s * 2)
                else:
                    c = math.sqrt((gamma + beta) / (gamma * 2))
                    s = p / (gamma * c * 2)
                a = b = 0.0
                for k in range(m):
                    t0 = c * At[i][k] + s * At[j][k]
                    t1 = -s * At[i][k] + c * At[j][k]
                    At[i][k], At[j][k] = t0, t1
                    a += t0 * t0
                    b += t1 * t1
                W[i], W[j] = a, b
                changed = True
                for k in range(n):
                    t0 = c * Vt[i][k] + s * Vt[j][k]
                    t1 = -s * Vt[i][k] + c * Vt[j][k]
                    Vt[i][k], Vt[j][k] = t0, t1
        if not changed:
            break
    W = [math.sqrt(sum_seq([t * t for t in At[i]])) for i in range(n)]
    for i in range(n - 1):
        j = i
        for k in range(i + 1, n):
            if W[j] < W[k]:
                j = k
        if i != j:
            W[i], W[j] = W[j], W[i]
            At[i], At[j] = At[j], At[i]
            Vt[i], Vt[j] = Vt[j], Vt[i]
    # zero singular values only feed rows that back-substitution skips; normalise the rest
    for i in range(n):
        if W[i] > np.finfo(np.float64).tiny:
            s = 1 / W[i]
            At[i] = [t * s for t in At[i]]
    thr = sum_seq(W) * (np.finfo(np.float64).eps * 2)
    x = [0.0] * n
    for i in range(n):
        wi = W[i]
        if abs(wi) <= thr:
            continue
        wi = 1 / wi
        s = sum_seq([At[i][j] * bv[j] for j in range(m)]) * wi
        x = [x[j] + s * Vt[i][j] for j in range(n)]
    return np.array(x + [1.0], dtype=np.float64).reshape(3, 3)


def sum_seq(vals):
    s = 0.0
    for v in vals:
        s += v
    return s


def invert3x3(M):
    m = [float(v) for v in np.asarray(M, dtype=np.float64).ravel()]
    def g(i, j):
        return m[i * 3 + j]
    d = (g(0, 0) * (g(1, 1) * g(2, 2) - g(1, 2) * g(2, 1)) - g(0, 1) * (g(1, 0) * g(2, 2) - g(1, 2) * g(2, 0))
         + g(0, 2) * (g(1, 0) * g(2, 1) - g(1, 1) * g(2, 0)))
    if d == 0.0:
        return np.zeros((3, 3))
    d = 1.0 / d
    t = [(g(1, 1) * g(2, 2) - g(1, 2) * g(2, 1)) * d, (g(0, 2) * g(2, 1) - g(0, 1) * g(2, 2)) * d,
         (g(0, 1) * g(1, 2) - g(0, 2) * g(1, 1)) * d, (g(1, 2) * g(2, 0) - g(1, 0) * g(2, 2)) * d,
         (g(0, 0) * g(2, 2) - g(0, 2) * g(2, 0)) * d, (g(0, 2) * g(1, 0) - g(0, 0) * g(1, 2)) * d,
         (g(1, 0) * g(2, 1) - g(1, 1) * g(2, 0)) * d, (g(0, 1) * g(2, 0) - g(0, 0) * g(2, 1)) * d,
         (g(0, 0) * g(1, 1) - g(0, 1) * g(1, 0)) * d]
    return np.array(t).reshape(3, 3)


def warp_perspective(src: np.ndarray, Minv: np.ndarray) -> np.ndarray:
    """warpPerspective with an already-inverted matrix (block origin xb, FP64, 1/32 px)."""
    h, w = src.shape
    M = np.asarray(Minv, dtype=np.float64).ravel()
    bh0 = min(16, h)
    bw0 = min(1024 // bh0, w)
    ys, xs = np.meshgrid(np.arange(h, dtype=np.float64), np.arange(w), indexing="ij")
    xb = (xs // bw0) * bw0
    x1 = (xs - xb).astype(np.float64)
    xb = xb.astype(np.float64)
    X0 = M[0] * xb + M[1] * ys + M[2]
    Y0 = M[3] * xb + M[4] * ys + M[5]
    W0 = M[6] * xb + M[7] * ys + M[8]
    Wd = W0 + M[6] * x1
    with np.errstate(divide="ignore"):
        Wd = np.where(Wd != 0, 32.0 / np.where(Wd != 0, Wd, 1.0), 0.0)
    fX = np.clip((X0 + M[0] * x1) * Wd, -2.0**31, 2.0**31 - 1)
    fY = np.clip((Y0 + M[3] * x1) * Wd, -2.0**31, 2.0**31 - 1)
    X = np.rint(fX).astype(np.int64)
    Y = np.rint(fY).astype(np.int64)
    sx = np.clip(X >> 5, -32768, 32767)
    sy = np.clip(Y >> 5, -32768, 32767)
    fx, fy = X & 31, Y & 31
    w0 = (32 - fx) * (32 - fy) * 32
    w1 = fx * (32 - fy) * 32
    w2 = (32 - fx) * fy * 32
    w3 = fx * fy * 32
    s = src.astype(np.int64)
    def tap(yy, xx):
        ok = (xx >= 0) & (xx < w) & (yy >= 0) & (yy < h)
        return np.where(ok, s[np.clip(yy, 0, h - 1), np.clip(xx, 0, w - 1)], 0)
    v = tap(sy, sx) * w0 + tap(sy, sx + 1) * w1 + tap(sy + 1, sx) * w2 + tap(sy + 1, sx + 1) * w3
    return np.clip((v + (1 << 14)) >> 15, 0, 255).astype(np.uint8)


def grid_points(w, h, ps):
    pts = [(i, j) for i in range(0, w, ps) for j in range(0, h, ps)]
    return np.array(pts, dtype=np.float32).reshape(-1, 2)


def calculate_optical_flow(img1, img2, pixel_step=10, min_vector_size=1.0, win=40, max_level=5,
                           thresh=190):
    """Whole path; returns dict(next_pts, status, vectors, num_vectors, H, Hinv, mask)."""
    g1, g2 = to_gray(img1), to_gray(img2)
    h, w = g1.shape
    pts = grid_points(w, h, pixel_step)
    p1, ml = build_pyramid(g1, win, max_level)
    p2, ml = build_pyramid(g2, win, ml)
    nextp, status = lk(p1, p2, ml, pts, win=win)
    vec = np.zeros((len(pts), 4))
    src, dst = [], []
    num = 0
    for i in range(len(pts)):
        sx, sy = pts[i]
        if status[i]:
            xd = np.float32(nextp[i, 0] - sx)
            yd = np.float32(nextp[i, 1] - sy)
            if abs(float(xd)) > min_vector_size or abs(float(yd)) > min_vector_size:
                vec[i] = (sx, sy, xd, yd)
                src.append(pts[i]); dst.append(nextp[i])
                num += 1
            else:
                vec[i] = (sx, sy, 0, 0)
        else:
            vec[i] = (-1, -1, 0, 0)
    out = dict(next_pts=nextp, status=status, vectors=vec, num_vectors=num,
               H=np.zeros((3, 3)), Hinv=np.zeros((3, 3)), mask=np.zeros_like(g1))
    if num >= 4:
        H = get_perspective_transform(src[:4], dst[:4])
        Hinv = invert3x3(H)
        warped = warp_perspective(g1, Hinv)
        d = np.abs(warped.astype(np.int16) - g2.astype(np.int16))
        out.update(H=H, Hinv=Hinv, mask=np.where(d > thresh, 255, 0).astype(np.uint8))
    return out
