"""Trajectory subspace RANSAC: OutlierDetector::fitSubspace,
reference common/src/outlier_detector.cpp:236-331.

CPU tests pin the oracle (oracle/mdx_oracle.c ora_fit_subspace) and the host generator:
  * both glibc rand() restatements (oracle ora_rand, product mdx_rand) equal this machine's libc
    rand() after srand(seed) -- the reference's sample stream (:17, :226);
  * meanSubtract against a numpy restatement of :200-221 (float32 sequential sums, y flip);
  * every hypothesis's residuals against an independent numpy restatement that builds Pnd the
    reference's way (I - U_d U_d^T from an SVD of the sample, :266-283) in float64, and the
    winner / inlier counts / outlier decisions equal;
  * the decisions equal a float32 restatement of the reference's arithmetic (Eigen is float) on
    data without near-threshold residuals;
  * a known answer: trajectories of two rigid motions (camera, one object) fit the
    4*num_motions-dim model, erratic ones (tracking failures) are the outliers.
GPU tests (-m gpu): mdx_fit_subspace (through the C-ABI) equals the oracle bit for bit (columns,
outlier flags, residuals as float64 bits, outlier points).
"""
import ctypes as C

import numpy as np
import pytest

P99 = [0.0, 0.020, 0.115, 0.297, 0.554, 0.872, 1.239, 1.646, 2.088, 2.558]


def scene_trajectories(n_bg=600, n_fg=80, T=5, seed=0, noise=0.05, n_bad=0):
    """Background points under a per-frame affine camera, a foreground object under its own
    translation (num_motions = 2 rigid motions), and n_bad erratic trajectories (a few px of
    random jump per frame: the tracking failures fitSubspace is meant to flag)."""
    rng = np.random.default_rng(seed)
    bg = rng.uniform([20, 20], [620, 460], (n_bg, 2))
    fg = rng.uniform([250, 180], [350, 260], (n_fg, 2))
    bad = rng.uniform([20, 20], [620, 460], (n_bad, 2))
    out = np.zeros((n_bg + n_fg + n_bad, T, 2))
    for t in range(T):
        a = np.radians(0.4 * t)
        A = 1.01 ** t * np.array([[np.cos(a), -np.sin(a)], [np.sin(a), np.cos(a)]])
        out[:n_bg, t] = bg @ A.T + np.array([2.5 * t, -1.2 * t])
        out[n_bg:n_bg + n_fg, t] = fg + np.array([-6.0 * t, 4.0 * t])
        out[n_bg + n_fg:, t] = bad + (rng.normal(0, 4.0, (n_bad, 2)) if t else 0.0)
    out += rng.normal(0, noise, out.shape)
    idx = rng.permutation(len(out))
    return out[idx].astype(np.float32), (idx >= n_bg + n_fg)


def np_mean_subtract(traj):
    traj = traj.astype(np.float32)
    N, T = traj.shape[:2]
    xs = np.float32(traj[0, 0, 0]); ys = np.float32(traj[0, 0, 1])
    for i in range(1, N):
        xs = np.float32(xs + traj[i, 0, 0]); ys = np.float32(ys + traj[i, 0, 1])
    xc, yc = np.float32(float(xs) / N), np.float32(float(ys) / N)
    d = traj.reshape(N, 2 * T).copy()
    d[:, 0::2] = d[:, 0::2] - xc
    d[:, 1::2] = yc - d[:, 1::2]
    return d


def np_fit_subspace(traj, num_motions, sigma, draws, dtype=np.float64):
    """Independent restatement of :236-331 with numpy's SVD; `draws` = the rand() stream."""
    data = np_mean_subtract(traj).astype(dtype).T          # n x N, column = trajectory
    n, N = data.shape
    d = 4 * num_motions
    best, best_res, best_cols, allres = 0, None, None, []
    for it in range(50):
        cols = [draws[it * d + k] % N for k in range(d)]
        U, _, _ = np.linalg.svd(data[:, cols], full_matrices=True)
        Pnd = np.eye(n, dtype=dtype) - U[:, :d] @ U[:, :d].T
        res = np.abs(np.einsum("ki,ki->i", data, Pnd @ data))
        allres.append(res)
        npts = int((res < (n - d) * sigma * sigma).sum())
        if npts > best:
            best, best_res, best_cols = npts, res, cols
    thr = sigma * sigma * P99[n - d] if 0 < n - d < 10 else 0.2
    out = np.zeros(N, np.uint8) if best_res is None else (best_res > thr).astype(np.uint8)
    return best_cols, out, best_res, allres


def _libc_draws(seed, k):
    libc = C.CDLL("libc.so.6")
    libc.srand(C.c_uint(seed))
    return [libc.rand() for _ in range(k)]


@pytest.mark.parametrize("seed", [0, 1, 12345, 2 ** 31 + 5, 2 ** 32 - 1, 20141105])
def test_rand_matches_libc(mdx, oracle, seed):
    ref = _libc_draws(seed, 5000)
    st = oracle.rand_state(seed)
    assert [oracle.rand(st) for _ in range(5000)] == ref
    ps = mdx._lib.MdxRandState()
    mdx.lib().mdx_srand(C.byref(ps), seed)
    assert [mdx.lib().mdx_rand(C.byref(ps)) for _ in range(5000)] == ref


def test_mean_subtract(oracle):
    traj, _ = scene_trajectories(seed=3)
    np.testing.assert_array_equal(oracle.subspace_data(traj), np_mean_subtract(traj))


@pytest.mark.parametrize("num_motions,T,sigma", [(2, 5, 0.5), (3, 7, 1.0), (2, 5, 4.0), (4, 9, 0.5)])
def test_oracle_matches_svd_restatement(oracle, num_motions, T, sigma):
    traj, _ = scene_trajectories(T=T, seed=num_motions + T)
    seed = 99 + T
    r = oracle.fit_subspace(traj, num_motions, sigma, oracle.rand_state(seed))
    draws = _libc_draws(seed, 50 * 4 * num_motions)
    cols, out, res, _ = np_fit_subspace(traj, num_motions, sigma, draws)
    assert list(r["columns"]) == cols
    np.testing.assert_allclose(r["residuals"], res, rtol=1e-6, atol=1e-9)
    np.testing.assert_array_equal(r["is_outlier"], out)
    assert r["n_outliers"] == int(out.sum())


def test_float32_reference_arithmetic_same_decisions(oracle):
    """The reference computes in float (Eigen::MatrixXf): on data whose residuals are not within
    float rounding of the thresholds the winner and outliers are the same."""
    traj, _ = scene_trajectories(seed=11, noise=0.02)
    r = oracle.fit_subspace(traj, 2, 0.5, oracle.rand_state(5))
    cols, out, res, _ = np_fit_subspace(traj, 2, 0.5, _libc_draws(5, 400), dtype=np.float32)
    thr = 0.25 * P99[2]
    near = np.abs(r["residuals"] - thr) < 1e-3 * max(thr, 1.0)
    assert list(r["columns"]) == cols
    assert np.array_equal(r["is_outlier"][~near], out[~near])


def test_float_mode_is_float_arithmetic(oracle):
    """precision 1 (explicit float Pnd, float x'(Pnd x), outlier_detector.cpp:272-290): residuals
    differ from the double mode's only by float rounding -- bounded by a few ulps of |x|^2 per
    term -- and the decisions agree away from the thresholds."""
    traj, _ = scene_trajectories(seed=11, noise=0.02)
    r64 = oracle.fit_subspace(traj, 2, 0.5, oracle.rand_state(5))
    r32 = oracle.fit_subspace(traj, 2, 0.5, oracle.rand_state(5), precision=1)
    assert list(r32["columns"]) == list(r64["columns"])
    data = oracle.subspace_data(traj).reshape(len(traj), -1).astype(np.float64)
    n = data.shape[1]
    tol = 8 * n * n * np.finfo(np.float32).eps * (data ** 2).sum(axis=1)
    diff = np.abs(r32["residuals"] - r64["residuals"])
    assert np.all(diff <= tol + 1e-6), float((diff / (tol + 1e-6)).max())
    assert np.any(diff > 0)                       # the float path really ran
    thr = 0.25 * P99[2]
    away = np.abs(r64["residuals"] - thr) > tol
    assert np.array_equal(r32["is_outlier"][away], r64["is_outlier"][away])


def test_known_answer_erratic_trajectories_are_outliers(oracle):
    """Two rigid motions (camera + one object) span the 4*num_motions = 8-dim model; erratic
    trajectories (tracking failures) fall outside it and are the outliers."""
    traj, bad = scene_trajectories(n_bg=800, n_fg=150, n_bad=40, seed=21, noise=0.03)
    r = oracle.fit_subspace(traj, 2, 1.0, oracle.rand_state(2))
    out = r["is_outlier"].astype(bool)
    assert out[bad].mean() > 0.9 and out[~bad].mean() < 0.02


def test_degenerate_arguments(oracle):
    traj = np.zeros((10, 5, 2), np.float32)
    assert oracle.fit_subspace(traj, 3, 0.5, oracle.rand_state(1))["n_outliers"] == -1   # d = 12 > n = 10
    assert oracle.fit_subspace(np.zeros((0, 5, 2), np.float32), 2, 0.5, oracle.rand_state(1))["n_outliers"] == -1


# ------------------------------------------------------------------------------------ GPU
def _gpu_vs_oracle(mdx, ctx, oracle, traj, num_motions, sigma, seed, precision=0):
    ps = mdx._lib.MdxRandState()
    mdx.lib().mdx_srand(C.byref(ps), seed)
    g = ctx.fit_subspace(traj, num_motions, sigma, ps)
    r = oracle.fit_subspace(traj, num_motions, sigma, oracle.rand_state(seed), precision)
    np.testing.assert_array_equal(g.columns, r["columns"])
    np.testing.assert_array_equal(g.is_outlier, r["is_outlier"])
    np.testing.assert_array_equal(g.residuals.view(np.uint64), r["residuals"].view(np.uint64))
    T = traj.shape[1]
    exp_pts = traj[r["is_outlier"].astype(bool), max(T - 2, 0)]
    np.testing.assert_array_equal(g.outlier_points, exp_pts)
    # the generator advanced exactly like the reference's: 50 x d draws
    st = oracle.rand_state(seed)
    for _ in range(50 * 4 * num_motions):
        oracle.rand(st)
    assert mdx.lib().mdx_rand(C.byref(ps)) == oracle.rand(st)
    return g


@pytest.mark.gpu
@pytest.mark.parametrize("n_bg,n_fg,T,nm,sigma,seed", [
    (600, 80, 5, 2, 0.5, 1), (3000, 400, 5, 2, 1.0, 2), (20000, 2000, 5, 2, 0.5, 7), (500, 60, 7, 3, 0.5, 3), (400, 50, 9, 4, 2.0, 4),
    (3, 0, 5, 2, 0.5, 5), (1, 0, 5, 2, 0.5, 6),
])
def test_subspace_gpu_bit_exact(mdx, ctx, oracle, n_bg, n_fg, T, nm, sigma, seed):
    traj, _ = scene_trajectories(n_bg=n_bg, n_fg=n_fg, T=T, seed=seed)
    _gpu_vs_oracle(mdx, ctx, oracle, traj, nm, sigma, seed)


@pytest.mark.gpu
@pytest.mark.parametrize("n_bg,n_fg,T,nm,sigma,seed", [
    (600, 80, 5, 2, 0.5, 1), (20000, 2000, 5, 2, 0.5, 7), (500, 60, 7, 3, 0.5, 3), (400, 50, 9, 4, 2.0, 4),
    (3, 0, 5, 2, 0.5, 5),
])
def test_subspace_gpu_float_mode_bit_exact(mdx, oracle, n_bg, n_fg, T, nm, sigma, seed):
    """MDX_SUBSPACE_F32 (the reference's float arithmetic shape): GPU == the oracle's float mode,
    residual bits included."""
    traj, _ = scene_trajectories(n_bg=n_bg, n_fg=n_fg, T=T, seed=seed)
    with mdx.Context(0, 64, 64, 1, subspace_precision=mdx.SUBSPACE_F32) as c:
        _gpu_vs_oracle(mdx, c, oracle, traj, nm, sigma, seed, precision=1)


@pytest.mark.gpu
def test_subspace_on_tracked_trajectories(mdx, ctx, oracle):
    """The node's chain (node.cpp:295-348): trajectories from mdx_flow_trajectory, then fitSubspace."""
    from traj_seq import sequence
    frames = sequence(mdx, oracle, 320, 240, 5, seed=12)
    res = ctx.flow_trajectory(frames)
    traj = np.ascontiguousarray(np.array(res.trajectories, np.float32))
    assert len(traj) > 100
    _gpu_vs_oracle(mdx, ctx, oracle, traj, 2, 0.5, 77)


@pytest.mark.gpu
def test_outlier_detector_interface(mdx, oracle):
    traj, _ = scene_trajectories(seed=8)
    od = mdx.OutlierDetector(seed=31)
    try:
        pts = []
        sub = od.fitSubspace(list(traj), pts, 2, 0.5)
        pts2 = []
        od.fitSubspace(list(traj), pts2, 2, 0.5)     # second call continues the stream
    finally:
        od.close()
    st = oracle.rand_state(31)
    r1 = oracle.fit_subspace(traj, 2, 0.5, st)
    r2 = oracle.fit_subspace(traj, 2, 0.5, st)
    assert [tuple(t.ravel()) for t in sub] == [tuple(traj[i].ravel()) for i in r1["columns"]]
    assert pts == [tuple(p) for p in traj[r1["is_outlier"].astype(bool), 3]]
    assert pts2 == [tuple(p) for p in traj[r2["is_outlier"].astype(bool), 3]]
