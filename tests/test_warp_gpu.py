"""GPU parity of the fused warp + absdiff + threshold kernel (rows A8-A10) over the geometries
and thresholds its fast path special-cases, through the C-ABI entry `mdx_warp_diff_dev`.

Reference: common/src/optical_flow_calculator.cpp:124-127 (warpPerspective, absdiff,
threshold(., 190, 255, THRESH_BINARY)).  The checker is the oracle's warp_perspective
(OpenCV 2.4 WarpPerspectiveInvoker restated) + numpy absdiff/threshold; the bar is bit-exact.

Cases: frame widths that are / are not multiples of the 128-px tile (partial reference blocks),
band-edge rows, homographies whose 1/32-px coordinates fall exactly on rounding ties
(translation by 1/64 px), flips (M0 < 0), zoom in/out (footprint larger than the LDS staging
buffer -> general path), projective and singular M, and thresholds -1, 0, 10, 190, 254, 255, 300.
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _rot(deg, s=1.0, tx=0.0, ty=0.0, cx=0.0, cy=0.0):
    c, si = math.cos(math.radians(deg)) * s, math.sin(math.radians(deg)) * s
    # rotate/scale about (cx, cy), then translate
    return np.array([[c, -si, cx - c * cx + si * cy + tx], [si, c, cy - si * cx - c * cy + ty], [0.0, 0.0, 1.0]])


def _H(kind, w, h, Ht):
    return {
        "true": Ht,
        "identity": np.eye(3),
        "tie_translation": np.array([[1.0, 0.0, 1.0 / 64], [0.0, 1.0, -3.0 / 64], [0.0, 0.0, 1.0]]),
        "tie_scale_half": np.array([[0.5, 0.0, 0.25 / 32], [0.0, 2.0, 0.0], [0.0, 0.0, 1.0]]),
        "rot5": _rot(5.0, 1.0, 2.3, -1.1, w / 2, h / 2),
        "flip_x": np.array([[-1.0, 0.0, w - 1.0 + 0.3], [0.0, 1.0, 0.7], [0.0, 0.0, 1.0]]),
        "zoom_in": _rot(0.0, 1.6, 0.0, 0.0, w / 2, h / 2),
        "zoom_out": _rot(0.0, 0.6, 0.0, 0.0, w / 2, h / 2),
        "far_away": np.array([[1.0, 0.0, -5000.0], [0.0, 1.0, 12.0], [0.0, 0.0, 1.0]]),
        "m8_not_pow2": np.array([[1.01, 0.002, 3.2], [-0.003, 0.99, -1.7], [0.0, 0.0, 1.3]]),
        "projective": np.array([[1.002, 0.013, -2.5], [-0.011, 0.995, 1.75], [2.1e-5, -1.3e-5, 1.0]]),
        "singular": np.zeros((3, 3)),
        # fixed-point screening (k_warp_fx): rows y = 32 mod 64 sit exactly on rounding ties
        # (X = 32 x + y / 64), the others 1/64 px away; and coordinates 2^-23 px past a tie
        "tie_rows": np.array([[1.0, 1.0 / 2048, 0.0], [0.0, 1.0, 0.0], [0.0, 0.0, 1.0]]),
        "near_tie": np.array([[1.0, 0.0, 0.5 / 32 + 2.0 ** -28], [0.0, 1.0, -0.5 / 32 - 2.0 ** -29], [0.0, 0.0, 1.0]]),
        "near_tie_rot": _rot(0.25, 1.0, 0.5 / 32 + 2.0 ** -27, 0.5 / 32 - 2.0 ** -26, w / 2, h / 2),
        # projective fast path (per-pixel W and 32 / W): perspective in x and y; a tiny perspective term
        # on a 1/64-px translation, so X sits within ~x^2 2^-35 px of a rounding tie (the division's
        # last bits decide); and a horizon (W = 0) inside the frame, where tiles fall back
        "proj_xy": np.array([[0.98, 0.021, 4.5], [-0.017, 1.01, -3.25], [-3.1e-5, 2.4e-5, 1.0]]),
        "proj_near_tie": np.linalg.inv(np.array([[1.0, 0.0, 1.0 / 64], [0.0, 1.0, -1.0 / 64],
                                                 [2.0 ** -40, 2.0 ** -41, 1.0]])),
        "proj_horizon": np.linalg.inv(np.array([[1.0, 0.0, 0.0], [0.0, 1.0, 0.0], [-1.0 / (0.6 * w), 0.0, 1.0]])),
    }[kind]


@pytest.fixture(scope="module")
def wctx(mdx):
    c = mdx.Context(0, 3840, 2160, 1)
    yield c
    c.close()


def _run(mdx, ctx, oracle, g1, g2, Hs, thresh):
    B, h, w = g1.shape
    Hb = np.ascontiguousarray(np.stack(Hs).astype(np.float64))
    ctx.set_params(thresh=thresh)
    d1, d2, dH, dM = (ctx.dev_alloc(x) for x in (g1.nbytes, g2.nbytes, Hb.nbytes, B * w * h))
    try:
        ctx.h2d(d1, g1); ctx.h2d(d2, g2); ctx.h2d(dH, Hb)
        ctx.warp_diff_dev(B, d1, d2, w, h, w, w * h, dH, dM)
        ctx.sync()
        out = np.empty((B, h, w), np.uint8)
        ctx.d2h(out, dM)
    finally:
        ctx.set_params(thresh=190)
        for p in (d1, d2, dH, dM):
            ctx.dev_free(p)
    for i in range(B):
        warped = oracle.warp_perspective(g1[i], oracle.invert3x3(Hb[i]), nthreads=8)
        ref = np.where(np.abs(warped.astype(np.int16) - g2[i].astype(np.int16)) > thresh, 255, 0).astype(np.uint8)
        bad = np.argwhere(out[i] != ref)
        assert bad.size == 0, f"pair {i}: {len(bad)} mask pixels differ, first (y, x) {bad[:4].tolist()}"


KINDS = ["true", "identity", "tie_translation", "tie_scale_half", "rot5", "flip_x", "zoom_in", "zoom_out",
         "far_away", "m8_not_pow2", "projective", "singular", "tie_rows", "near_tie", "near_tie_rot", "proj_xy",
         "proj_near_tie", "proj_horizon"]


@pytest.mark.parametrize("w,h", [(640, 480), (1000, 300), (1984, 70), (128, 64), (132, 65), (68, 33)])
def test_warp_geometries(mdx, wctx, oracle, w, h):
    g1, g2 = [], []
    Hs = []
    for i, kind in enumerate(KINDS):
        a, b, Ht = mdx.synth_pair(500 + i, w, h, 1)
        g1.append(a); g2.append(b)
        Hs.append(_H(kind, w, h, Ht))
    _run(mdx, wctx, oracle, np.stack(g1), np.stack(g2), Hs, 190)


@pytest.mark.parametrize("thresh", [-1, 0, 10, 190, 254, 255, 300])
def test_warp_thresholds(mdx, wctx, oracle, thresh):
    w, h = 640, 480
    a, b, Ht = mdx.synth_pair(77, w, h, 1)
    a2, b2, _ = mdx.synth_pair(78, w, h, 1)
    _run(mdx, wctx, oracle, np.stack([a, a2]), np.stack([b, b2]), [Ht, _H("rot5", w, h, Ht)], thresh)


def test_warp_4k_true_h(mdx, wctx, oracle):
    """The roofline workload's geometry (bench.py --only-roofline), one pair."""
    w, h = 3840, 2160
    a, b, Ht = mdx.synth_pair(20141105, w, h, 1)
    _run(mdx, wctx, oracle, a[None], b[None], [Ht], 190)


def test_warp_4k_projective(mdx, wctx, oracle):
    """The bench's projective roofline sub-line geometry (roofline.projective): 4K with the tests'
    perspective H, and its near-tie variant, both on the projective fast path."""
    w, h = 3840, 2160
    a, b, Ht = mdx.synth_pair(20141105, w, h, 1)
    a2, b2, _ = mdx.synth_pair(20141106, w, h, 1)
    _run(mdx, wctx, oracle, np.stack([a, a2]), np.stack([b, b2]),
         [_H("projective", w, h, Ht), _H("proj_near_tie", w, h, Ht)], 190)


def test_warp_projective_random(mdx, wctx, oracle):
    """Random projective H across the projective fast path's range (round 6: one v_rcp_f64 per four
    pixels of the product of their W, one quadratic Newton step, the shift-add boundary test):
    perspective terms from 1e-7 to 4e-4 per pixel, rotations, anisotropic scales and translations
    with 1/64-px parts, every mask byte against the oracle.  The first eight stay mild (|angle| <=
    1 deg, scales 0.97-1.03, perspective <= 5e-5: W within ~10% over the frame), so nearly every
    tile's footprint fits the staging buffer and takes the projective fast path; the last four are
    strong (W varying by up to ~1.5x, a horizon in some), where tiles also fall back."""
    w, h = 1920, 1080
    rng = np.random.default_rng(20261018)
    g1, g2, Hs = [], [], []
    for i in range(12):
        a, b, _ = mdx.synth_pair(900 + i, w, h, 1)
        g1.append(a); g2.append(b)
        mild = i < 8
        ang = math.radians(rng.uniform(-1.0, 1.0) if mild else rng.uniform(-8.0, 8.0))
        sx, sy = rng.uniform(0.97, 1.03, 2) if mild else rng.uniform(0.8, 1.25, 2)
        p6, p7 = (rng.choice([-1.0, 1.0], 2) * 10.0 ** rng.uniform(-7.0, -4.3 if mild else -3.4, 2))
        tx, ty = rng.uniform(-30, 30, 2) + rng.integers(0, 64, 2) / 64.0
        Hs.append(np.array([[sx * math.cos(ang), -sy * math.sin(ang), tx],
                            [sx * math.sin(ang), sy * math.cos(ang), ty], [p6, p7, 1.0]]))
    _run(mdx, wctx, oracle, np.stack(g1), np.stack(g2), Hs, 190)


def test_div32_is_ieee_division(mdx, wctx):
    """The projective fast path's 32 / W (mdx_warp.hip div32: the IEEE division sequence without its
    range-scaling steps) equals correctly rounded IEEE division bit for bit over its range
    |W| in [2^-100, 2^100]: random mantissas over every exponent, both signs, and hard mantissas
    (all ones, powers of two, near one)."""
    import ctypes as C
    rng = np.random.default_rng(11)
    n = 1 << 20
    e = rng.integers(-100, 100, n)
    m = 1.0 + rng.random(n)
    d = np.ldexp(m, e) * np.where(rng.random(n) < 0.5, -1.0, 1.0)
    hard = []
    for ex in range(-100, 100):
        for mm in (1.0, np.nextafter(2.0, 0.0), np.nextafter(1.0, 2.0), 1.5, 1.0 + 2.0 ** -26, 2.0 - 2.0 ** -26):
            hard += [np.ldexp(mm, ex), -np.ldexp(mm, ex)]
    d[:len(hard)] = hard
    d = np.ascontiguousarray(d[(np.abs(d) >= 2.0 ** -100) & (np.abs(d) <= 2.0 ** 100)])
    di, do = wctx.dev_alloc(d.nbytes), wctx.dev_alloc(d.nbytes)
    try:
        wctx.h2d(di, d)
        assert mdx.lib().mdx_debug_div32(wctx._h, C.c_void_p(di), C.c_void_p(do), len(d)) == 0
        wctx.sync()
        out = np.empty_like(d)
        wctx.d2h(out, do)
    finally:
        wctx.dev_free(di)
        wctx.dev_free(do)
    ref = 32.0 / d
    bad = np.nonzero(out.view(np.uint64) != ref.view(np.uint64))[0]
    assert bad.size == 0, f"{bad.size} of {len(d)} differ, first W {d[bad[:4]].tolist()}"


def test_copy_ceiling_probe(mdx, wctx):
    """The bench's copy-ceiling probe (mdx_probe_stream3_dev) computes the same 3 B/px result as an
    identity warp would: mask = |a - b| > t; and rejects unaligned sizes."""
    rng = np.random.default_rng(5)
    n = 1 << 20
    a = rng.integers(0, 256, n, dtype=np.uint8)
    b = rng.integers(0, 256, n, dtype=np.uint8)
    da, db, dm = (wctx.dev_alloc(n) for _ in range(3))
    try:
        wctx.h2d(da, a); wctx.h2d(db, b)
        for t in (-1, 0, 190, 255):
            wctx.probe_stream3_dev(n, da, db, dm, t)
            wctx.sync()
            out = np.empty(n, np.uint8)
            wctx.d2h(out, dm)
            ref = np.where(np.abs(a.astype(np.int16) - b.astype(np.int16)) > t, 255, 0).astype(np.uint8)
            assert np.array_equal(out, ref), t
        with pytest.raises(mdx.MdxError):
            wctx.probe_stream3_dev(n - 8, da, db, dm)
    finally:
        for p in (da, db, dm):
            wctx.dev_free(p)
