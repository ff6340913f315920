"""CPU checks of the oracle (oracle/mdx_oracle.c via oracle/pyoracle.py).

The oracle is test infrastructure: a C restatement of the OpenCV 2.4 semantics that
OpticalFlowCalculator::calculateOpticalFlow (reference common/src/optical_flow_calculator.cpp:30-130)
relies on.  The reference ships no tests or fixtures and OpenCV is absent here,
so the oracle is pinned by (1) the committed golden vectors, (2) an independently written numpy
restatement (tests/np_reference.py), and (3) known-answer tests whose results follow from the
OpenCV formulas by hand.  Parity with a real OpenCV 2.4 binary remains unpinned.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import np_reference as npr

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def _golden_names():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return sorted(json.load(f))


@pytest.mark.parametrize("simd", [False, True], ids=["scalar", "sse2"])
@pytest.mark.parametrize("name", _golden_names())
def test_oracle_matches_golden(oracle, name, simd):
    """Both oracle modes (the scalar C loops and the SSE2 restatement timed as the CPU baseline)
    reproduce every committed golden vector."""
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        man = json.load(f)[name]
    g = np.load(os.path.join(GOLDEN, name + ".npz"))
    assert _sha(g["img1"], g["img2"]) == man["inputs_sha256"]
    r = oracle.calculate_optical_flow(g["img1"], g["img2"], pixel_step=int(g["pixel_step"]),
                                      min_vector_size=float(g["min_vector_size"]), simd=simd)
    assert r["num_vectors"] == int(g["num_vectors"]) == man["num_vectors"]
    assert np.array_equal(r["status"], g["status"])
    assert np.array_equal(r["next_pts"].view(np.uint32), g["next_pts"].view(np.uint32))
    assert np.array_equal(r["vectors"], g["vectors"])
    assert np.array_equal(r["H"], g["H"])
    assert np.array_equal(r["mask"], g["mask"])
    assert _sha(r["next_pts"], r["status"], r["vectors"], r["mask"], r["H"]) == man["outputs_sha256"]


def _scene(seed, w, h, channels=1):
    """Small seeded scene for the numpy cross-check: blurred noise + rectangles, frame 2 shifted."""
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, (h + 16, w + 16, channels)).astype(np.float64)
    k = np.array([1, 4, 6, 4, 1], float) / 16
    for ax in (0, 1):
        base = np.apply_along_axis(lambda v: np.convolve(v, k, "same"), ax, base)
    base = np.clip((base - base.mean()) * 3 + 128, 0, 255)
    for _ in range(4):
        x0, y0 = rng.integers(0, w), rng.integers(0, h)
        base[y0:y0 + h // 5, x0:x0 + w // 5] = rng.integers(0, 256)
    dx, dy = int(rng.integers(-3, 4)), int(rng.integers(-3, 4))
    a = base[8:8 + h, 8:8 + w].astype(np.uint8)
    b = base[8 + dy:8 + dy + h, 8 + dx:8 + dx + w].astype(np.uint8)
    if channels == 1:
        a, b = a[..., 0], b[..., 0]
    return np.ascontiguousarray(a), np.ascontiguousarray(b)


@pytest.mark.parametrize("seed,w,h,ps,ch", [(1, 64, 48, 6, 1), (2, 90, 70, 5, 1), (3, 80, 60, 7, 3), (4, 50, 41, 4, 1)])
def test_oracle_matches_numpy_restatement(oracle, seed, w, h, ps, ch):
    a, b = _scene(seed, w, h, ch)
    r = oracle.calculate_optical_flow(a, b, pixel_step=ps, min_vector_size=0.5)
    c = npr.calculate_optical_flow(a, b, pixel_step=ps, min_vector_size=0.5)
    assert r["num_vectors"] == c["num_vectors"]
    assert np.array_equal(r["status"], c["status"])
    assert np.array_equal(r["next_pts"].view(np.uint32), c["next_pts"].view(np.uint32))
    assert np.array_equal(r["vectors"], c["vectors"])
    assert np.array_equal(r["H"], c["H"])
    assert np.array_equal(r["mask"], c["mask"])


@pytest.mark.parametrize("w,h,ps,ch,seed", [(1920, 1080, 10, 1, 20141105), (1920, 1080, 10, 1, 20141108),
                                             (640, 480, 3, 3, 7), (333, 241, 7, 1, 11), (81, 83, 1, 1, 31)])
def test_sse2_oracle_equals_scalar(oracle, w, h, ps, ch, seed):
    """The SSE2 restatement (oracle/mdx_oracle_sse2.c; OpenCV 2.4's x86 lane order) against the
    scalar loops, bit for bit, on the bench's 1080p pairs and other geometries: the CPU baseline
    times the same arithmetic the GPU is checked against."""
    import motion_detection_amd as m
    a, b, _ = m.synth_pair(seed, w, h, ch, 8)
    r = oracle.calculate_optical_flow(a, b, nthreads=8, pixel_step=ps, min_vector_size=1.0)
    s = oracle.calculate_optical_flow(a, b, nthreads=8, pixel_step=ps, min_vector_size=1.0, simd=True)
    assert r["num_vectors"] == s["num_vectors"]
    for k in ("next_pts", "status", "vectors", "H", "mask"):
        assert np.array_equal(np.asarray(r[k]).view(np.uint8), np.asarray(s[k]).view(np.uint8)), k


# ---------------------------------------------------------------- known-answer tests

def test_gray_conversion_weights(oracle):
    # cvtColor(CV_BGR2GRAY) on rgb8 data (optical_flow_calculator.cpp:50): R gets the B weight
    rgb = np.zeros((2, 3, 3), np.uint8)
    rgb[0, 0] = (255, 0, 0)
    rgb[0, 1] = (0, 255, 0)
    rgb[0, 2] = (0, 0, 255)
    rgb[1, :] = (77, 77, 77)
    g = oracle.to_gray(rgb)
    assert g[0, 0] == (255 * 1868 + 8192) >> 14        # 29: R weighted as blue
    assert g[0, 1] == (255 * 9617 + 8192) >> 14        # 150
    assert g[0, 2] == (255 * 4899 + 8192) >> 14        # 76: B weighted as red
    assert np.all(g[1] == 77)                          # grey replicated -> identity
    assert np.array_equal(g, npr.to_gray(rgb))


@pytest.mark.parametrize("v", [0, 1, 77, 255])
def test_pyrdown_constant(oracle, v):
    src = np.full((37, 53), v, np.uint8)
    d = oracle.pyrdown(src)
    assert d.shape == (19, 27)
    assert np.all(d == v)


def test_pyrdown_matches_numpy(oracle):
    rng = np.random.default_rng(5)
    for (h, w) in [(8, 8), (9, 13), (31, 2), (64, 97)]:
        src = rng.integers(0, 256, (h, w)).astype(np.uint8)
        assert np.array_equal(oracle.pyrdown(src), npr.pyrdown(src))


def test_scharr_constant_and_ramp(oracle):
    assert np.all(oracle.scharr(np.full((20, 30), 123, np.uint8)) == 0)
    # horizontal ramp v = 3x: interior Ix = (3+10+3) * (v[x+1] - v[x-1]) = 16 * 6 = 96, Iy = 0
    ramp = np.tile((3 * np.arange(40)).astype(np.uint8), (16, 1))
    d = oracle.scharr(ramp)
    assert np.all(d[:, 1:-1, 0] == 96)
    assert np.all(d[..., 1] == 0)
    # reflect-101 border: x=0 sees v[1] on both sides -> Ix = 0
    assert np.all(d[:, 0, 0] == 0)
    assert np.array_equal(d, npr.scharr(ramp))


def test_pyramid_levels_follow_win_rule(oracle):
    # buildOpticalFlowPyramid stops when the next level's side <= win (SURVEY.md §8 level table)
    for (w, h, levels) in [(640, 480, 4), (1920, 1080, 5), (160, 120, 2), (81, 81, 2), (80, 80, 1)]:
        ml, imgs, _ = oracle.build_pyramid(np.zeros((h, w), np.uint8), win=40, max_level=5, with_deriv=False)
        assert ml + 1 == len(imgs) == levels, (w, h, ml)


def test_warp_identity_and_translation(oracle):
    rng = np.random.default_rng(9)
    src = rng.integers(0, 256, (50, 70)).astype(np.uint8)
    assert np.array_equal(oracle.warp_perspective(src, np.eye(3)), src)
    # dst(x, y) = src(x + 3, y - 2) via the inverse map Minv; out-of-range taps -> 0
    Minv = np.array([[1, 0, 3], [0, 1, -2], [0, 0, 1]], float)
    out = oracle.warp_perspective(src, Minv)
    exp = np.zeros_like(src)
    exp[2:, :-3] = src[:-2, 3:]
    assert np.array_equal(out, exp)
    assert np.array_equal(out, npr.warp_perspective(src, Minv))


def test_perspective_fit_recovers_homography(oracle):
    H = np.array([[1.01, 0.02, 3.2], [-0.015, 0.99, -1.7], [1e-5, -2e-5, 1.0]])
    src = np.array([[10, 12], [300, 20], [280, 200], [15, 190]], float)
    p = np.c_[src, np.ones(4)] @ H.T
    dst = p[:, :2] / p[:, 2:]
    M = oracle.get_perspective_transform(src.astype(np.float32), dst.astype(np.float32))
    assert np.allclose(M, H, rtol=1e-4, atol=1e-6)


def test_collinear_first4_gives_constant_warp(oracle):
    """First-4 fit on points of column x=0 (the reference's usual case): the DLT
    has zero columns, M is singular, its inverse is all-zero and the warp is gray1(0, 0)."""
    src = np.array([[0, 0], [0, 10], [0, 20], [0, 30]], np.float32)
    dst = src + np.float32([1.5, -0.5])
    M = oracle.get_perspective_transform(src, dst)
    assert M[0, 0] == 0 and M[1, 0] == 0 and M[2, 0] == 0
    Minv = oracle.invert3x3(M)
    assert np.all(Minv == 0)
    img = np.random.default_rng(3).integers(0, 256, (30, 40)).astype(np.uint8)
    assert np.all(oracle.warp_perspective(img, Minv) == img[0, 0])


@pytest.mark.parametrize("eps,iters,tol", [(0.03, 10, 0.03), (1e-4, 40, 2e-3)])
def test_lk_integer_translation(oracle, eps, iters, tol):
    """1-px integer translation: every confidently tracked point moves by (1, 0).  The Newton
    loop stops once |delta| <= eps, so the residual is bounded by eps (reference: 0.03, :44);
    with a tight eps the tracker converges to the true shift."""
    rng = np.random.default_rng(11)
    base = rng.integers(0, 256, (140, 200)).astype(np.float64)
    k = np.array([1, 4, 6, 4, 1], float) / 16
    for ax in (0, 1):
        base = np.apply_along_axis(lambda v: np.convolve(v, k, "same"), ax, base)
    img = np.clip(base * 2 - 128, 0, 255).astype(np.uint8)
    a = np.ascontiguousarray(img[20:120, 20:180])
    b = np.ascontiguousarray(img[20:120, 19:179])          # content moves +1 px in x
    r = oracle.calculate_optical_flow(a, b, pixel_step=10, min_vector_size=0.5, eps=eps, max_iters=iters)
    n = oracle.grid_count(160, 100, 10)
    pts = npr.grid_points(160, 100, 10)
    inner = (pts[:, 0] >= 30) & (pts[:, 0] <= 130) & (pts[:, 1] >= 30) & (pts[:, 1] <= 70)
    ok = (r["status"] == 1) & inner
    assert ok.sum() > 20
    d = r["next_pts"][ok] - pts[ok]
    assert np.all(np.abs(d - [1.0, 0.0]) < tol)
    assert r["next_pts"].shape == (n, 2)


def test_flat_scene_has_no_vectors(oracle):
    f = np.full((64, 80), 90, np.uint8)
    r = oracle.calculate_optical_flow(f, f, pixel_step=8, min_vector_size=1.0)
    assert r["num_vectors"] == 0
    assert np.all(r["status"] == 0)                       # minEig < 1e-3 everywhere
    assert np.all(r["vectors"][:, :2] == -1)
    assert np.all(r["mask"] == 0)


def test_grid_order_is_x_major(oracle):
    pts = npr.grid_points(25, 17, 10)
    assert oracle.grid_count(25, 17, 10) == len(pts) == 3 * 2
    assert pts[:3].tolist() == [[0, 0], [0, 10], [10, 0]]


def test_svd_vblas_reading_sensitivity(oracle):
    """OpenCV 2.4's JacobiSVDImpl_ under CV_SSE2 may route the column dot products and norms
    through VBLAS<double>::dot / givensx (two-lane partial sums).  Both readings are valid SVD
    solves; this pins how far apart they leave getPerspectiveTransform: the
    matrices agree to 1e-9 relative, and the share of bit-different entries is recorded."""
    rng = np.random.default_rng(11)
    diff = total = 0
    worst = 0.0
    try:
        for t in range(400):
            if t % 4 == 0:   # the reference's usual case: four points of column x = 0 (collinear)
                src = np.array([[0, 10 * i] for i in range(4)], np.float32)
            else:
                src = rng.uniform(0, 1920, (4, 2)).astype(np.float32)
            dst = (src + rng.normal(0, 3, (4, 2))).astype(np.float32)
            oracle.set_svd_vblas(False)
            M0 = oracle.get_perspective_transform(src, dst)
            oracle.set_svd_vblas(True)
            M1 = oracle.get_perspective_transform(src, dst)
            total += 9
            diff += int((M0.view(np.uint64) != M1.view(np.uint64)).sum())
            scale = np.maximum(np.abs(M0), 1e-300)
            worst = max(worst, float(np.max(np.abs(M1 - M0) / np.maximum(scale, 1.0))))
    finally:
        oracle.set_svd_vblas(False)
    print(f"VBLAS reading: {diff} of {total} H entries bit-different, worst relative {worst:.3g}")
    assert worst < 1e-9
