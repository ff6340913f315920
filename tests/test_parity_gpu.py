"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle, bit for bit.

Bar: LK output points are compared as float32 bit patterns and must be
identical (the kernel reproduces the reference's SSE2 summation order), status / Vec4d
vectors / num_vectors / H / mask must be identical too.  The north-star tolerance
(1e-4 relative on flow) is therefore met with margin 0.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _compare(res, ref, label=""):
    assert res.num_vectors == ref["num_vectors"], label
    np.testing.assert_array_equal(res.status, ref["status"], err_msg=label)
    bad = np.nonzero(res.next_pts.view(np.uint32) != ref["next_pts"].view(np.uint32))[0]
    assert bad.size == 0, f"{label}: {bad.size} LK points differ, first {bad[:5]}: " \
                          f"{res.next_pts[bad[:3]]} vs {ref['next_pts'][bad[:3]]}"
    np.testing.assert_array_equal(res.vectors, ref["vectors"], err_msg=label)
    np.testing.assert_array_equal(res.H.view(np.uint64), ref["H"].view(np.uint64), err_msg=label)
    if res.mask is not None:
        nbad = int((res.mask != ref["mask"]).sum())
        assert nbad == 0, f"{label}: {nbad} mask pixels differ"


CASES = [
    # (w, h, pixel_step, channels, seed)
    (160, 120, 10, 1, 1),
    (640, 480, 10, 1, 20141105),
    (640, 480, 3, 1, 7),
    (333, 241, 7, 1, 11),
    (320, 240, 10, 3, 5),
    (1920, 1080, 10, 1, 20141106),
    # dense and sparse grids, frames at the pyramid's 40-px limits: pixel_step 1 (every pixel a
    # point, the step where the reference's Vec4d writes overflow), 2, 4, 16, 40, 64
    (81, 83, 1, 1, 31),
    (41, 41, 1, 1, 36),
    (64, 41, 2, 1, 32),
    (200, 150, 4, 1, 33),
    (200, 150, 16, 1, 34),
    (210, 160, 40, 1, 35),
    (1920, 1080, 64, 1, 37),
]


@pytest.mark.parametrize("w,h,ps,ch,seed", CASES)
def test_full_path_bit_exact(mdx, ctx, oracle, w, h, ps, ch, seed):
    a, b, _ = mdx.synth_pair(seed, w, h, ch)
    ctx.set_params(pixel_step=ps, min_vector_size=1.0, fit_mode=mdx.FIT_FIRST4)
    res = ctx.flow_warp_diff(a, b)
    ref = oracle.calculate_optical_flow(a, b, nthreads=8, pixel_step=ps, min_vector_size=1.0)
    _compare(res, ref, f"{w}x{h} ps{ps} ch{ch}")


def test_bgr_input(mdx, ctx, oracle):
    a, b, _ = mdx.synth_pair(3, 320, 240, 3)
    ctx.set_params(pixel_step=10, min_vector_size=0.4, fit_mode=mdx.FIT_FIRST4)
    res = ctx.flow_warp_diff(a, b, fmt=mdx.FMT_BGR8)
    ref = oracle.calculate_optical_flow(a, b, fmt=oracle.FMT_BGR8, pixel_step=10, min_vector_size=0.4)
    _compare(res, ref, "bgr8")


def test_translation_known_answer(mdx, ctx, oracle):
    """Integer translation of a textured scene: flow == shift to LK precision, bit-exact vs oracle."""
    big, _, _ = mdx.synth_pair(99, 400, 300, 1)
    a = np.ascontiguousarray(big[20:260, 20:340])
    b = np.ascontiguousarray(big[17:257, 15:335])   # scene moves by (+5, +3)
    ctx.set_params(pixel_step=10, min_vector_size=1.0, fit_mode=mdx.FIT_FIRST4)
    res = ctx.flow_warp_diff(a, b)
    ref = oracle.calculate_optical_flow(a, b, pixel_step=10)
    _compare(res, ref, "translation")
    d = res.next_pts - mdx.grid_points(320, 240, 10)
    inner = (res.status == 1)
    med = np.median(d[inner], axis=0)
    assert abs(med[0] - 5) < 0.05 and abs(med[1] - 3) < 0.05


def test_flat_frames_no_vectors(mdx, ctx, oracle):
    """Constant frames: every minEig test fails -> status 0, no vectors, no mask (:118)."""
    a = np.full((120, 160), 77, np.uint8)
    ctx.set_params(pixel_step=10, fit_mode=mdx.FIT_FIRST4)
    res = ctx.flow_warp_diff(a, a.copy())
    ref = oracle.calculate_optical_flow(a, a.copy(), pixel_step=10)
    assert res.num_vectors == 0 and res.code == mdx.MDX_EDEGENERATE
    assert res.status.sum() == 0
    _compare(res, ref, "flat")
    assert res.mask.max() == 0


def test_identical_frames(mdx, ctx, oracle):
    a, _, _ = mdx.synth_pair(4, 200, 150, 1)
    res = ctx.flow_warp_diff(a, a.copy())
    ref = oracle.calculate_optical_flow(a, a.copy(), pixel_step=ctx.params.pixel_step)
    _compare(res, ref, "identical")


@pytest.mark.parametrize("w,h", [(48, 48), (41, 90), (63, 45), (81, 81)])
def test_small_frames(mdx, ctx, oracle, w, h):
    """Single-level pyramids, widths below the 64-px warp block, reflect-101 multi-folds."""
    a, b, _ = mdx.synth_pair(w * 1000 + h, w, h, 1)
    ctx.set_params(pixel_step=5, min_vector_size=1.0, fit_mode=mdx.FIT_FIRST4)
    res = ctx.flow_warp_diff(a, b)
    ref = oracle.calculate_optical_flow(a, b, pixel_step=5)
    _compare(res, ref, f"{w}x{h}")


def _projective(w, h):
    return np.array([[1.002, 0.013, -2.5], [-0.011, 0.995, 1.75], [2.1e-5, -1.3e-5, 1.0]])


@pytest.mark.parametrize("kind", ["true_affine", "projective", "singular"])
def test_external_h_warp(mdx, ctx, oracle, kind):
    w, h = 640, 480
    a, b, Ht = mdx.synth_pair(21, w, h, 1)
    H = {"true_affine": Ht, "projective": _projective(w, h), "singular": np.zeros((3, 3))}[kind]
    ctx.set_params(pixel_step=10, fit_mode=mdx.FIT_EXTERNAL)
    try:
        res = ctx.flow_warp_diff(a, b, H_external=H)
    finally:
        ctx.set_params(fit_mode=mdx.FIT_FIRST4)
    Hinv = oracle.invert3x3(H)
    warped = oracle.warp_perspective(a, Hinv)
    d = np.abs(warped.astype(np.int16) - b.astype(np.int16))
    ref_mask = np.where(d > 190, 255, 0).astype(np.uint8)
    assert int((res.mask != ref_mask).sum()) == 0
    np.testing.assert_array_equal(res.H, H)


def test_warp_diff_dev_batch(mdx, ctx, oracle):
    """The standalone fused warp+diff entry over a batch with per-pair H (roofline kernel)."""
    w, h, B = 500, 300, 3
    frames1, frames2, Hs = [], [], []
    for i in range(B):
        a, b, Ht = mdx.synth_pair(100 + i, w, h, 1)
        frames1.append(a); frames2.append(b)
        Hs.append(Ht if i != 1 else _projective(w, h))
    g1 = np.stack(frames1); g2 = np.stack(frames2); Hb = np.stack(Hs).astype(np.float64)
    d1, d2, dH, dM = (ctx.dev_alloc(x) for x in (g1.nbytes, g2.nbytes, Hb.nbytes, B * w * h))
    try:
        ctx.h2d(d1, g1); ctx.h2d(d2, g2); ctx.h2d(dH, Hb)
        ctx.warp_diff_dev(B, d1, d2, w, h, w, w * h, dH, dM)
        ctx.sync()
        out = np.empty((B, h, w), np.uint8)
        ctx.d2h(out, dM)
    finally:
        for p in (d1, d2, dH, dM):
            ctx.dev_free(p)
    for i in range(B):
        warped = oracle.warp_perspective(g1[i], oracle.invert3x3(Hb[i]))
        ref = np.where(np.abs(warped.astype(np.int16) - g2[i].astype(np.int16)) > 190, 255, 0).astype(np.uint8)
        assert int((out[i] != ref).sum()) == 0, f"pair {i}"


@pytest.mark.parametrize("B,env,wh", [
    (4, {}, (320, 240)),
    # 11 pairs: the LK queue's 8 per-XCD ranges split pairs; sub-batches of 3; both group sizes
    (11, {"MDX_LK_SUB": "3"}, (320, 240)),
    (11, {"MDX_LK_G": "4"}, (320, 240)),
    (11, {"MDX_LK_G": "8"}, (320, 240)),
    (5, {"MDX_LK_AUX": "0"}, (320, 240)),   # class / A kernels on the main stream
    # LK dataflow (batch a multiple of 8 and >= 16, npts a multiple of 16): level l-1's launch
    # overlaps level l's and waits per pair; per sub-batch; off; group size 8 everywhere; a larger
    # frame; 24 pairs (three per XCD)
    (16, {}, (320, 240)),
    (32, {"MDX_LK_SUB": "16"}, (320, 240)),
    (24, {}, (320, 240)),
    (16, {"MDX_LK_FLOW": "0"}, (320, 240)),
    (16, {"MDX_LK_G": "8"}, (320, 240)),
    (16, {}, (640, 480)),
])
def test_batch_dev_matches_host_path(mdx, oracle, monkeypatch, B, env, wh):
    """The zero-copy batched entry gives the same per-pair results as the oracle."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    w, h = wh
    pairs = [mdx.synth_pair(300 + i, w, h, 1) for i in range(B)]
    g1 = np.stack([p[0] for p in pairs]); g2 = np.stack([p[1] for p in pairs])
    n = mdx.grid_count(w, h, 10)
    with mdx.Context(0, w, h, B) as c:
        c.set_params(pixel_step=10)
        bufs = {k: c.dev_alloc(s) for k, s in dict(i1=g1.nbytes, i2=g2.nbytes, np=B * n * 8, st=B * n,
                                                    vec=B * n * 32, mask=B * w * h, H=B * 72, num=B * 4).items()}
        c.h2d(bufs["i1"], g1); c.h2d(bufs["i2"], g2)
        c.flow_warp_diff_batch_dev(B, bufs["i1"], bufs["i2"], w, h, w, w * h, mdx.FMT_GRAY8, bufs["np"], bufs["st"],
                                   bufs["vec"], bufs["mask"], bufs["H"], 0, bufs["num"])
        c.sync()
        out = dict(np=np.empty((B, n, 2), np.float32), st=np.empty((B, n), np.uint8), vec=np.empty((B, n, 4)),
                   mask=np.empty((B, h, w), np.uint8), H=np.empty((B, 3, 3)), num=np.empty(B, np.int32))
        for k, arr in out.items():
            c.d2h(arr, bufs[k])
        for p in bufs.values():
            c.dev_free(p)
    for i in range(B):
        ref = oracle.calculate_optical_flow(g1[i], g2[i], pixel_step=10)
        assert out["num"][i] == ref["num_vectors"]
        np.testing.assert_array_equal(out["st"][i], ref["status"])
        np.testing.assert_array_equal(out["np"][i].view(np.uint32), ref["next_pts"].view(np.uint32))
        np.testing.assert_array_equal(out["vec"][i], ref["vectors"])
        np.testing.assert_array_equal(out["mask"][i], ref["mask"])
        np.testing.assert_array_equal(out["H"][i], ref["H"])


@pytest.mark.parametrize("w,h", [(320, 240), (640, 480)])
def test_batch_with_unfit_pair(mdx, oracle, w, h):
    """A pair with no fit (flat frames) between fitted pairs of one batch: its mask is written all
    zero (over a garbage-filled buffer) and the neighbours match the oracle.  k_warp_diff reads
    every tile's TileInfo before testing the pair's fit status; an unfit pair's entries are never
    written by k_warp_prep, and must stay unused."""
    B = 3
    pairs = [mdx.synth_pair(700 + i, w, h, 1) for i in range(B)]
    flat = np.full((h, w), 77, np.uint8)
    g1 = np.stack([pairs[0][0], flat, pairs[2][0]]); g2 = np.stack([pairs[0][1], flat.copy(), pairs[2][1]])
    n = mdx.grid_count(w, h, 10)
    with mdx.Context(0, w, h, B) as c:
        c.set_params(pixel_step=10)
        bufs = {k: c.dev_alloc(s) for k, s in dict(i1=g1.nbytes, i2=g2.nbytes, np=B * n * 8, st=B * n,
                                                    vec=B * n * 32, mask=B * w * h, H=B * 72, num=B * 4).items()}
        c.h2d(bufs["i1"], g1); c.h2d(bufs["i2"], g2)
        c.h2d(bufs["mask"], np.full((B, h, w), 0xAB, np.uint8))
        c.flow_warp_diff_batch_dev(B, bufs["i1"], bufs["i2"], w, h, w, w * h, mdx.FMT_GRAY8, bufs["np"], bufs["st"],
                                   bufs["vec"], bufs["mask"], bufs["H"], 0, bufs["num"])
        c.sync()
        mask = np.empty((B, h, w), np.uint8); num = np.empty(B, np.int32)
        c.d2h(mask, bufs["mask"]); c.d2h(num, bufs["num"])
        for p in bufs.values():
            c.dev_free(p)
    assert num[1] == 0 and mask[1].max() == 0
    for i in (0, 2):
        ref = oracle.calculate_optical_flow(g1[i], g2[i], pixel_step=10)
        assert num[i] == ref["num_vectors"] >= 4
        np.testing.assert_array_equal(mask[i], ref["mask"])


def test_reference_interface(mdx, oracle):
    """OpticalFlowCalculator.calculateOpticalFlow fills the vector Mat and comp like the reference."""
    a, b, _ = mdx.synth_pair(8, 320, 240, 3)
    ofc = mdx.OpticalFlowCalculator(max_w=320, max_h=240)
    vec = np.zeros((240, 320, 4))
    comp = np.zeros((240, 320), np.uint8)
    num = ofc.calculateOpticalFlow(a, b, vec, 10, comp, 1.0)
    ref = oracle.calculate_optical_flow(a, b, pixel_step=10, min_vector_size=1.0)
    assert num == ref["num_vectors"]
    pts = mdx.grid_points(320, 240, 10).astype(int)
    np.testing.assert_array_equal(vec[pts[:, 1], pts[:, 0]], ref["vectors"])
    np.testing.assert_array_equal(comp, ref["mask"])
    ofc.close()


@pytest.mark.parametrize("w,h,ps,nb,ch,pipe", [(640, 480, 10, 3, 1, "0"), (333, 241, 7, 5, 1, "0"),
                                               (1920, 1080, 10, 8, 1, "0"), (640, 480, 3, 2, 3, "0"),
                                               (320, 240, 10, 1, 1, "0"), (7680, 4320, 10, 8, 3, "0"),
                                               (640, 480, 3, 2, 3, "1"), (1920, 1080, 10, 8, 1, "1")])
def test_row_tiled_matches_full(mdx, monkeypatch, w, h, ps, nb, ch, pipe):
    """Row bands run one after another on one GPU, records exchanged through
    host memory: every point, the fit, the count and every mask row equal the full path's (also
    with call pipelining, whose band calls alternate pyramid halves)."""
    from motion_detection_amd import rowtile
    a, b, _ = mdx.synth_pair(7000 + nb, w, h, ch)
    fmt = mdx.FMT_GRAY8 if ch == 1 else mdx.FMT_RGB8
    with mdx.Context(0, w, h, 1, pixel_step=ps, min_vector_size=1.0, call_pipelining=int(pipe)) as c:
        full = c.flow_warp_diff(a, b, fmt=fmt)
        n = mdx.grid_count(w, h, ps)
        stride = w * ch
        d = {k: c.dev_alloc(sz) for k, sz in dict(i1=a.nbytes, i2=b.nbytes, np=n * 8, st=n, vec=n * 32,
                                                   cand=nb * 96, mask=w * h, H=72, num=4).items()}
        try:
            c.h2d(d["i1"], a); c.h2d(d["i2"], b)
            zero = np.zeros(n * 32, np.uint8)
            c.h2d(d["vec"], zero)
            for r in range(nb):
                y0, y1 = rowtile.band_rows(h, nb, r)
                c.band_flow_dev(d["i1"], d["i2"], w, h, stride, fmt, y0, y1, d["np"], d["st"], d["cand"] + 96 * r,
                                d["vec"])
            recs = np.empty(nb, rowtile.BAND_CAND_DTYPE)
            c.sync()
            c.d2h(recs, d["cand"])
            for r in range(nb):
                y0, y1 = rowtile.band_rows(h, nb, r)
                c.band_fit_warp_dev(nb, d["cand"], y0, y1, d["mask"] + y0 * w, d["H"], d["num"])
            c.sync()
            out = dict(np=np.empty((n, 2), np.float32), st=np.empty(n, np.uint8), vec=np.empty((n, 4)),
                       mask=np.empty((h, w), np.uint8), H=np.empty((3, 3)), num=np.empty(1, np.int32))
            for k, arr in out.items():
                c.d2h(arr, d[k])
        finally:
            for p in d.values():
                c.dev_free(p)
    np.testing.assert_array_equal(out["st"], full.status)
    np.testing.assert_array_equal(out["np"].view(np.uint32), full.next_pts.view(np.uint32))
    np.testing.assert_array_equal(out["vec"], full.vectors)
    assert int(out["num"][0]) == full.num_vectors == int(recs["count"].sum())
    np.testing.assert_array_equal(out["H"].view(np.uint64), full.H.view(np.uint64))
    assert int((out["mask"] != full.mask).sum()) == 0


def _fit_cases(n, seed):
    """First-4 correspondences for the fit alone: random quads, one grid column (the typical first-4
    pick, collinear sources), a repeated point, all-zero destinations, 8K-scale coordinates."""
    rng = np.random.default_rng(seed)
    src = np.empty((n, 4, 2), np.float32)
    dst = np.empty((n, 4, 2), np.float32)
    for c in range(n):
        kind = c % 5
        scale = 7680 if kind == 4 else 1920
        s = (10 * rng.integers(0, scale // 10, (4, 2))).astype(np.float32)
        if kind == 1:
            s[:, 0] = s[0, 0]
            s[:, 1] = 10 * rng.integers(0, 100) + 10 * np.arange(4)
        if kind == 2:
            s[3] = s[0]
        d = (s + rng.uniform(-3, 3, (4, 2))).astype(np.float32)
        if kind == 3:
            d[:] = 0
        src[c], dst[c] = s, d
    return src, dst


def test_fit_arbitrary_correspondences(mdx, oracle):
    """k_band_fit's wave-parallel JacobiSVD fit (the same solve as k_fit) on 250 arbitrary
    first-4 correspondences, fed through the band API's records: H equals the oracle's
    getPerspectiveTransform bit for bit, degenerate inputs included (collinear, repeated, zero)."""
    from motion_detection_amd import rowtile
    w, h, ps, n = 320, 240, 10, 250
    src, dst = _fit_cases(n, 20261018)
    a, b, _ = mdx.synth_pair(9, w, h, 1)
    npts = mdx.grid_count(w, h, ps)
    recs = np.zeros(n, rowtile.BAND_CAND_DTYPE)
    recs["count"] = 4
    recs["n"] = 4
    recs["idx"] = np.arange(4)
    recs["src"] = src.reshape(n, 8)
    recs["dst"] = dst.reshape(n, 8)
    with mdx.Context(0, w, h, 1, pixel_step=ps, min_vector_size=1.0) as c:
        d = {k: c.dev_alloc(sz) for k, sz in dict(i1=a.nbytes, i2=b.nbytes, np=npts * 8, st=npts, cand=96,
                                                   cands=n * 96, mask=w * h, H=n * 72).items()}
        try:
            c.h2d(d["i1"], a); c.h2d(d["i2"], b)
            c.band_flow_dev(d["i1"], d["i2"], w, h, w, mdx.FMT_GRAY8, 0, h, d["np"], d["st"], d["cand"])
            c.h2d(d["cands"], recs)
            for i in range(n):        # record i alone: its four points are the first four overall
                c.band_fit_warp_dev(1, d["cands"] + 96 * i, 0, h, d["mask"], d["H"] + 72 * i)
            c.sync()
            H = np.empty((n, 9))
            c.d2h(H, d["H"])
        finally:
            for p in d.values():
                c.dev_free(p)
    bad = [i for i in range(n)
           if not np.array_equal(H[i].view(np.uint64), oracle.get_perspective_transform(src[i], dst[i]).ravel().view(np.uint64))]
    assert not bad, f"{len(bad)} of {n} fits differ, first {bad[:5]}"


@pytest.mark.parametrize("B,uniq,pipe", [(2, 2, 0), (8, 4, 1)])
def test_full_path_4k_bit_exact(mdx, oracle, B, uniq, pipe):
    """Config C2 (3840x2160, 5 pyramid levels) through the batched device entry: every output
    equals the oracle's.  (8, 4, 1) is the bench's full_path_4k leg exactly: 8 slots holding 4
    distinct pairs, call pipelining on, the same call made twice back to back without a sync."""
    w, h = 3840, 2160
    uniq_pairs = [mdx.synth_pair(40 + i, w, h, 1) for i in range(uniq)]
    pairs = [uniq_pairs[i % uniq] for i in range(B)]
    g1 = np.stack([p[0] for p in pairs]); g2 = np.stack([p[1] for p in pairs])
    n = mdx.grid_count(w, h, 10)
    with mdx.Context(0, w, h, B, pixel_step=10, min_vector_size=1.0, call_pipelining=pipe) as c:
        bufs = [c.dev_alloc(x) for x in (g1.nbytes, g2.nbytes, B * n * 8, B * n, B * n * 32, B * w * h, B * 72, B * 4)]
        try:
            c.h2d(bufs[0], g1); c.h2d(bufs[1], g2)
            for _ in range(1 + pipe):
                c.flow_warp_diff_batch_dev(B, bufs[0], bufs[1], w, h, w, w * h, mdx.FMT_GRAY8, d_next_pts=bufs[2],
                                           d_status=bufs[3], d_vectors=bufs[4], d_mask=bufs[5], d_H=bufs[6],
                                           d_num_vectors=bufs[7])
            c.sync()
            npts = np.empty((B, n, 2), np.float32); st = np.empty((B, n), np.uint8)
            vec = np.empty((B, n, 4)); mask = np.empty((B, h, w), np.uint8)
            H = np.empty((B, 9)); num = np.empty(B, np.int32)
            for arr, p in zip((npts, st, vec, mask, H, num), bufs[2:]):
                c.d2h(arr, p)
        finally:
            for p in bufs:
                c.dev_free(p)
    refs = [oracle.calculate_optical_flow(a, b, nthreads=16, pixel_step=10, min_vector_size=1.0)
            for a, b, _ in uniq_pairs]
    for i in range(B):
        ref = refs[i % uniq]
        assert num[i] == ref["num_vectors"]
        np.testing.assert_array_equal(st[i], ref["status"])
        np.testing.assert_array_equal(npts[i].view(np.uint32), ref["next_pts"].view(np.uint32))
        np.testing.assert_array_equal(vec[i], ref["vectors"])
        np.testing.assert_array_equal(H[i].view(np.uint64), ref["H"].ravel().view(np.uint64))
        assert int((mask[i] != ref["mask"]).sum()) == 0, f"pair {i}"


def test_full_path_8k_rgb_bit_exact(mdx, oracle):
    """Config C4's frame (7680x4320 rgb8, 6 pyramid levels 0..5) on one GPU: every output equals
    the oracle's (the row-tiled form is checked against this path above)."""
    w, h = 7680, 4320
    a, b, _ = mdx.synth_pair(4242, w, h, 3)
    with mdx.Context(0, w, h, 1, pixel_step=10, min_vector_size=1.0) as c:
        res = c.flow_warp_diff(a, b, fmt=mdx.FMT_RGB8)
    ref = oracle.calculate_optical_flow(a, b, fmt=oracle.FMT_RGB8, nthreads=16, pixel_step=10, min_vector_size=1.0)
    _compare(res, ref, "8k rgb")


@pytest.mark.parametrize("pipe", [1, 0])
def test_back_to_back_calls_pipelined(mdx, oracle, pipe):
    """Calls enqueued back to back without a host sync (the bench's pattern): with call pipelining
    (mdx_params.call_pipelining, inputs resident before each call) each call's front end runs beside
    the previous call's last level and fit/warp, on the other half of the pyramid slabs.  Four calls
    on three different batches into separate outputs, a synchronous trajectory call in between:
    every call's results equal the oracle's."""
    w, h, B = 320, 240, 8
    n = mdx.grid_count(w, h, 10)
    sets = [[mdx.synth_pair(700 + 10 * s + i, w, h, 1) for i in range(B)] for s in range(3)]
    order = [0, 1, 2, 0]
    with mdx.Context(0, w, h, B, call_pipelining=pipe) as c:
        c.set_params(pixel_step=10)
        ins = []
        for pairs in sets:
            g1 = np.stack([p[0] for p in pairs]); g2 = np.stack([p[1] for p in pairs])
            d1, d2 = c.dev_alloc(g1.nbytes), c.dev_alloc(g2.nbytes)
            c.h2d(d1, g1); c.h2d(d2, g2)
            ins.append((d1, d2))
        outs = [{k: c.dev_alloc(s) for k, s in dict(np=B * n * 8, st=B * n, mask=B * w * h, num=B * 4).items()}
                for _ in order]
        for j, si in enumerate(order):
            d1, d2 = ins[si]
            o = outs[j]
            c.flow_warp_diff_batch_dev(B, d1, d2, w, h, w, w * h, mdx.FMT_GRAY8, o["np"], o["st"], 0, o["mask"], 0, 0,
                                       o["num"])
            if j == 1:   # a synchronous entry on the shared slabs between pipelined calls
                seq = [sets[2][0][0], sets[2][0][1], sets[2][1][0]]
                tr = c.flow_trajectory(seq)
                ref_tr = oracle.flow_trajectory(seq, pixel_step=10)
                assert tr.num_vectors == ref_tr["num_vectors"]
        c.sync()
        got = []
        for o in outs:
            r = dict(np=np.empty((B, n, 2), np.float32), st=np.empty((B, n), np.uint8),
                     mask=np.empty((B, h, w), np.uint8), num=np.empty(B, np.int32))
            for k, arr in r.items():
                c.d2h(arr, o[k])
            got.append(r)
        for o in outs:
            for p in o.values():
                c.dev_free(p)
        for d1, d2 in ins:
            c.dev_free(d1); c.dev_free(d2)
    for j, si in enumerate(order):
        for i in range(B):
            ref = oracle.calculate_optical_flow(sets[si][i][0], sets[si][i][1], pixel_step=10)
            assert got[j]["num"][i] == ref["num_vectors"], (j, i)
            np.testing.assert_array_equal(got[j]["st"][i], ref["status"])
            np.testing.assert_array_equal(got[j]["np"][i].view(np.uint32), ref["next_pts"].view(np.uint32))
            np.testing.assert_array_equal(got[j]["mask"][i], ref["mask"])


@pytest.mark.parametrize("w,h,ps,nb,ch,pipe", [(640, 480, 10, 4, 1, "0"), (1280, 720, 7, 3, 3, "0"),
                                               (640, 480, 10, 4, 1, "1")])
def test_row_bands_on_separate_contexts(mdx, monkeypatch, w, h, ps, nb, ch, pipe):
    """Each band on its own context, as on its own GPU: a band's flow builds frame 1's pyramid for
    its rows only, so the rows its warp reads beyond the band (camera motion) come from the frame
    at fit/warp time.  Every mask row equals the full path's (also with call pipelining)."""
    from motion_detection_amd import rowtile
    a, b, _ = mdx.synth_pair(7100 + nb, w, h, ch)
    fmt = mdx.FMT_GRAY8 if ch == 1 else mdx.FMT_RGB8
    n = mdx.grid_count(w, h, ps)
    ctxs = [mdx.Context(0, w, h, 1, pixel_step=ps, min_vector_size=1.0, call_pipelining=int(pipe)) for _ in range(nb)]
    try:
        full = ctxs[0].flow_warp_diff(a, b, fmt=fmt)
        recs = np.empty(nb, rowtile.BAND_CAND_DTYPE)
        bufs = []
        for r, c in enumerate(ctxs):
            d = {k: c.dev_alloc(sz) for k, sz in dict(i1=a.nbytes, i2=b.nbytes, np=n * 8, st=n, cand=96,
                                                       cands=nb * 96, mask=w * h, num=4).items()}
            c.h2d(d["i1"], a); c.h2d(d["i2"], b)
            y0, y1 = rowtile.band_rows(h, nb, r)
            c.band_flow_dev(d["i1"], d["i2"], w, h, w * ch, fmt, y0, y1, d["np"], d["st"], d["cand"])
            c.sync()
            one = np.empty(1, rowtile.BAND_CAND_DTYPE)
            c.d2h(one, d["cand"])
            recs[r] = one[0]
            bufs.append(d)
        mask = np.empty((h, w), np.uint8)
        for r, (c, d) in enumerate(zip(ctxs, bufs)):
            y0, y1 = rowtile.band_rows(h, nb, r)
            c.h2d(d["cands"], recs.view(np.uint8))
            c.band_fit_warp_dev(nb, d["cands"], y0, y1, d["mask"], 0, d["num"])
            c.sync()
            band = np.empty((y1 - y0, w), np.uint8)
            c.d2h(band, d["mask"])
            mask[y0:y1] = band
        for c, d in zip(ctxs, bufs):
            for p in d.values():
                c.dev_free(p)
    finally:
        for c in ctxs:
            c.close()
    assert int((mask != full.mask).sum()) == 0
