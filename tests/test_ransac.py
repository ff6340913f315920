"""MDX_FIT_RANSAC: the deterministic RANSAC homography option (include/mdx.h).  NOT in the reference
-- its fit is getPerspectiveTransform on the first four accepted vectors
(common/src/optical_flow_calculator.cpp:118-120), which MDX_FIT_FIRST4 keeps -- so parity with the
reference is N/A; this option follows north_star's "RANSAC global-motion fit" wording, with every
hypothesis solved by the reference's own 4-point solver.

CPU: the oracle's restatement (ora_fit_ransac) against an independent numpy restatement of the
draws and the inlier scoring, and known answers (an exact homography among outliers is found; on
the synthetic pair the fit recovers the generator's true motion, which the first-4 rule does not).
GPU: the k_ransac_* kernels equal the oracle bit for bit (H as float64 bits, num_vectors, mask).
"""
import numpy as np
import pytest

M64 = (1 << 64) - 1


def _mix64(z):
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def _np_ransac(oracle, src, dst, iters, thresh, seed):
    """Independent restatement: Python-int splitmix64 draws, numpy FP64 scoring (same evaluation
    order), the oracle's 4-point solver for each sample."""
    n = len(src)
    s64, d64 = src.astype(np.float64), dst.astype(np.float64)
    t2 = thresh * thresh
    best = (-1, 0, None)
    for h in range(iters):
        idx = []
        for j in range(4):
            c = 0
            while True:
                v = _mix64((seed << 32) | (h << 20) | (j << 16) | (c & 0xFFFF)) % n
                if v not in idx or c >= 0xFFFF:
                    idx.append(v)
                    break
                c += 1
        H = oracle.get_perspective_transform(src[idx], dst[idx]).ravel()
        sx, sy, dx, dy = s64[:, 0], s64[:, 1], d64[:, 0], d64[:, 1]
        nx = H[0] * sx + H[1] * sy + H[2]
        ny = H[3] * sx + H[4] * sy + H[5]
        dd = H[6] * sx + H[7] * sy + H[8]
        ex, ey = nx - dx * dd, ny - dy * dd
        cnt = int(np.count_nonzero(ex * ex + ey * ey <= t2 * (dd * dd)))
        if cnt > best[0]:
            best = (cnt, h, H.reshape(3, 3))
    return best


def _scene(n=400, outliers=0.3, seed=3):
    rng = np.random.default_rng(seed)
    H0 = np.array([[1.01, 0.02, 3.0], [-0.015, 0.99, -2.0], [1e-5, -2e-5, 1.0]])
    src = rng.uniform(0, 640, (n, 2)).astype(np.float32)
    p = np.c_[src.astype(np.float64), np.ones(n)] @ H0.T
    dst = (p[:, :2] / p[:, 2:]).astype(np.float32)
    bad = rng.random(n) < outliers
    dst[bad] += rng.uniform(-40, 40, (int(bad.sum()), 2)).astype(np.float32)
    return src, dst, H0, bad


def test_oracle_ransac_equals_numpy_restatement(oracle):
    src, dst, _, _ = _scene(300)
    for iters, thresh, seed in ((16, 3.0, 20141105), (40, 1.5, 7)):
        H, cnt, bh = oracle.fit_ransac(src, dst, iters, thresh, seed)
        rc, rh, rH = _np_ransac(oracle, src, dst, iters, thresh, seed)
        assert (cnt, bh) == (rc, rh)
        np.testing.assert_array_equal(H.view(np.uint64), rH.view(np.uint64))


def test_oracle_ransac_finds_the_homography_among_outliers(oracle):
    src, dst, H0, bad = _scene(500, 0.35)
    H, cnt, _ = oracle.fit_ransac(src, dst, 128, 3.0)
    assert cnt >= int((~bad).sum())                  # every true inlier (float-rounded dst) counted
    np.testing.assert_allclose(H / H[2, 2], H0, rtol=1e-3, atol=1e-5)
    H4, c4, _ = oracle.fit_ransac(src[:3], dst[:3], 8, 3.0)
    assert c4 == -1                                  # fewer than 4 vectors: no fit


def test_oracle_whole_path_ransac_recovers_true_motion(mdx, oracle):
    """On the synthetic pair (affine camera motion + a moving patch) RANSAC recovers H_true, while
    the reference's first-4 rule fits four collinear points of column x = 0 (singular M)."""
    a, b, Ht = mdx.synth_pair(20141105, 640, 480, 1)
    r = oracle.calculate_optical_flow(a, b, pixel_step=10, min_vector_size=1.0, fit_mode=2)
    f4 = oracle.calculate_optical_flow(a, b, pixel_step=10, min_vector_size=1.0)
    assert r["fit_status"] == 0 and r["num_vectors"] == f4["num_vectors"]
    xs, ys = np.meshgrid(np.arange(0, 640, 10), np.arange(0, 480, 10))
    P = np.c_[xs.ravel(), ys.ravel(), np.ones(xs.size)]

    def proj(H):
        q = P @ H.T
        return q[:, :2] / q[:, 2:]
    err = np.linalg.norm(proj(r["H"]) - proj(Ht), axis=1)
    assert np.median(err) < 1.0 and err.max() < 4.0   # one 4-point hypothesis, no refit
    assert abs(np.linalg.det(f4["Hinv"])) == 0.0      # first-4: singular, constant warp
    assert (r["mask"] > 0).mean() < 0.01              # the compensated difference is quiet


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,batch,iters,thresh,seed", [(640, 480, 4, 128, 3.0, 20141105),
                                                         (1920, 1080, 3, 64, 1.0, 99),
                                                         (320, 240, 2, 1000, 3.0, 5)])
def test_ransac_gpu_bit_exact(mdx, oracle, w, h, batch, iters, thresh, seed):
    pairs = [mdx.synth_pair(700 + i, w, h, 1, 16) for i in range(batch)]
    g1 = np.stack([p[0] for p in pairs])
    g2 = np.stack([p[1] for p in pairs])
    n = mdx.grid_count(w, h, 10)
    kw = dict(pixel_step=10, min_vector_size=1.0, fit_mode=2, ransac_iters=iters, ransac_thresh=thresh,
              ransac_seed=seed)
    with mdx.Context(0, w, h, batch, **kw) as c:
        d1, d2 = c.dev_alloc(g1.nbytes), c.dev_alloc(g2.nbytes)
        o = {k: c.dev_alloc(sz) for k, sz in dict(np=batch * n * 8, st=batch * n, mask=batch * w * h, H=batch * 72,
                                                  num=batch * 4).items()}
        c.h2d(d1, g1)
        c.h2d(d2, g2)
        c.flow_warp_diff_batch_dev(batch, d1, d2, w, h, w, w * h, 0, d_next_pts=o["np"], d_status=o["st"],
                                   d_mask=o["mask"], d_H=o["H"], d_num_vectors=o["num"])
        c.sync()
        H = np.empty((batch, 9))
        num = np.empty(batch, np.int32)
        mask = np.empty((batch, h, w), np.uint8)
        c.d2h(H, o["H"])
        c.d2h(num, o["num"])
        c.d2h(mask, o["mask"])
        # the host entry too (one pair)
        single = c.flow_warp_diff(g1[0], g2[0])
        for p in list(o.values()) + [d1, d2]:
            c.dev_free(p)
    for i, (a, b, _) in enumerate(pairs):
        ref = oracle.calculate_optical_flow(a, b, nthreads=16, ransac_iters=iters, ransac_thresh=thresh,
                                            ransac_seed=seed, **{k: v for k, v in kw.items() if not k.startswith("ransac")})
        assert num[i] == ref["num_vectors"]
        np.testing.assert_array_equal(H[i].view(np.uint64), ref["H"].ravel().view(np.uint64), err_msg=f"pair {i}")
        assert int((mask[i] != ref["mask"]).sum()) == 0, f"pair {i}"
        if i == 0:
            np.testing.assert_array_equal(single.H.ravel().view(np.uint64), ref["H"].ravel().view(np.uint64))
            assert np.array_equal(single.mask, ref["mask"])


def test_ransac_params_are_checked(mdx):
    p = mdx.default_params()
    assert (p.ransac_iters, p.ransac_thresh, p.ransac_seed) == (128, 3.0, 20141105)
    assert mdx.FIT_RANSAC == 2
