"""Trajectory tracking: calculateOpticalFlowTrajectory,
reference common/src/optical_flow_calculator.cpp:133-257.

CPU tests pin the oracle's restatement (oracle/mdx_oracle.c ora_flow_trajectory):
  * its per-point bookkeeping against an independent Python restatement of :143-249 driven by the
    oracle's per-pair LK (pyoracle.lk), bit for bit;
  * known answers: an integer camera translation is tracked to the translation within the LK's
    eps, points that would leave the 10-px border stay put and lose their trajectory, a flat
    scene tracks nothing.
GPU tests (-m gpu) compare mdx_flow_trajectory (through the C-ABI) with the oracle bit for bit:
trajectories (float32 bits), their lengths, the last pass's start points and Vec4d, num_vectors.
"""
import numpy as np
import pytest

from traj_seq import sequence


def _py_trajectory(oracle, frames, pixel_step, min_vector_size):
    """Independent restatement of optical_flow_calculator.cpp:143-249 over pyoracle.lk."""
    h, w = frames[0].shape[:2]
    gray = [oracle.to_gray(f) for f in frames]
    pts = np.array([(x, y) for x in range(0, w, pixel_step) for y in range(0, h, pixel_step)], np.float32)
    trajs = [[tuple(p)] for p in pts]
    vec = np.zeros((len(pts), 4))
    start = np.zeros((len(pts), 2), np.float32)
    num = 0
    for j in range(len(frames) - 1):
        last = j == len(frames) - 2
        nxt, st = oracle.lk(gray[j], gray[j + 1], pts)
        temp = pts.copy()
        for i in range(len(pts)):
            sx, sy = pts[i]
            if last:
                start[i] = pts[i]
            if st[i]:
                ex, ey = nxt[i]
                if last:
                    xd, yd = np.float32(ex - sx), np.float32(ey - sy)
                    if abs(float(xd)) > min_vector_size or abs(float(yd)) > min_vector_size:
                        vec[i] = (sx, sy, xd, yd)
                        num += 1
                    else:
                        vec[i] = (sx, sy, 0.0, 0.0)
                if ex > 10.0 and ey > 10.0 and ex < w - 10 and ey < h - 10:
                    temp[i] = nxt[i]
                    trajs[i].append((ex, ey))
            elif last:
                vec[i] = (-1.0, -1.0, 0.0, 0.0)
        pts = temp
    return num, trajs, start, vec


@pytest.mark.parametrize("w,h,n,ps,ch", [(160, 120, 5, 10, 1), (200, 150, 3, 7, 3), (96, 80, 4, 5, 1)])
def test_oracle_bookkeeping_matches_restatement(mdx, oracle, w, h, n, ps, ch):
    frames = sequence(mdx, oracle, w, h, n, seed=w + n, channels=ch)
    r = oracle.flow_trajectory(frames, pixel_step=ps, min_vector_size=1.0)
    num, trajs, start, vec = _py_trajectory(oracle, frames, ps, 1.0)
    assert r["num_vectors"] == num
    np.testing.assert_array_equal(r["traj_len"], [len(t) for t in trajs])
    for i, t in enumerate(trajs):
        np.testing.assert_array_equal(r["traj"][i, :len(t)], np.array(t, np.float32))
    np.testing.assert_array_equal(r["start_pts"], start)
    np.testing.assert_array_equal(r["vectors"], vec)
    assert len(r["trajectories"]) == sum(len(t) == n for t in trajs)


def test_integer_translation_tracked(mdx, oracle):
    """Camera translation of (+2, +1) px per frame: every complete trajectory advances by (2, 1)
    per frame to within the LK's stopping eps (0.03 px per step, TermCriteria :141)."""
    w, h, n = 160, 120, 5
    base, _, _ = mdx.synth_pair(3, w, h, 1)
    frames = [np.ascontiguousarray(np.roll(np.roll(base, 2 * k, axis=1), k, axis=0)) for k in range(n)]
    r = oracle.flow_trajectory(frames, pixel_step=10)
    full = np.array(r["trajectories"])
    assert len(full) > 0.5 * len(r["traj_len"])
    steps = np.diff(full, axis=1)
    assert np.abs(steps[..., 0] - 2.0).max() < 0.1 and np.abs(steps[..., 1] - 1.0).max() < 0.1
    # the last pass's vectors: |dx| = 2 > min_vector_size for every tracked point
    tracked = r["vectors"][:, 0] >= 0
    assert r["num_vectors"] == int(tracked.sum())


def test_border_points_stay(mdx, oracle):
    """A point whose tracked position is not strictly inside the 10-px border keeps its position
    and its trajectory stops growing (:207-216)."""
    w, h, n = 160, 120, 3
    base, _, _ = mdx.synth_pair(5, w, h, 1)
    frames = [np.ascontiguousarray(np.roll(base, 3 * k, axis=1)) for k in range(n)]
    r = oracle.flow_trajectory(frames, pixel_step=10)
    x0 = r["traj"][:, 0, 0]
    # grid points at x = 0 (and the columns the shift pushes past w-10) never extend
    assert np.all(r["traj_len"][x0 == 0] == 1)
    assert np.all(r["traj_len"][x0 >= w - 10] == 1)
    inner = (x0 >= 20) & (x0 <= w - 30) & (r["traj"][:, 0, 1] >= 20) & (r["traj"][:, 0, 1] <= h - 20)
    assert np.all(r["traj_len"][inner] == n)


def test_flat_scene_tracks_nothing(oracle):
    frames = [np.full((90, 120), 77, np.uint8)] * 3
    r = oracle.flow_trajectory(frames, pixel_step=10)
    assert r["num_vectors"] == 0 and r["trajectories"] == []
    assert np.all(r["vectors"][:, :2] == -1.0)


# ------------------------------------------------------------------------------------ GPU
GPU_CASES = [
    # (w, h, nimg, pixel_step, channels, seed)
    (320, 240, 5, 10, 1, 1),
    (320, 240, 5, 10, 3, 2),
    (640, 480, 3, 7, 1, 3),
    (200, 150, 2, 5, 1, 4),
    (1280, 720, 5, 10, 3, 5),
    # the chained launch at its frame limit (16), and past it (the per-pass launches)
    (200, 150, 16, 10, 1, 6),
    (160, 120, 18, 9, 1, 7),
]


def _compare(res, ref, label):
    assert res.num_vectors == ref["num_vectors"], label
    np.testing.assert_array_equal(res.traj_len, ref["traj_len"], err_msg=label)
    for i in range(len(res.traj_len)):
        k = int(ref["traj_len"][i])
        a, b = res.traj[i, :k].view(np.uint32), ref["traj"][i, :k].view(np.uint32)
        assert np.array_equal(a, b), f"{label}: point {i}: {res.traj[i, :k]} vs {ref['traj'][i, :k]}"
    np.testing.assert_array_equal(res.start_pts.view(np.uint32), ref["start_pts"].view(np.uint32), err_msg=label)
    np.testing.assert_array_equal(res.vectors.view(np.uint64), ref["vectors"].view(np.uint64), err_msg=label)


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,n,ps,ch,seed", GPU_CASES)
def test_trajectory_gpu_bit_exact(mdx, ctx, oracle, w, h, n, ps, ch, seed):
    frames = sequence(mdx, oracle, w, h, n, seed=seed, channels=ch)
    ctx.set_params(pixel_step=ps)
    try:
        res = ctx.flow_trajectory(frames)
    finally:
        ctx.set_params(pixel_step=10)
    ref = oracle.flow_trajectory(frames, pixel_step=ps, nthreads=8)
    _compare(res, ref, f"{w}x{h}x{n} ps{ps} ch{ch}")
    assert len(res.trajectories) == len(ref["trajectories"])


@pytest.mark.gpu
def test_trajectory_reference_interface(mdx, oracle):
    """OpticalFlowCalculator.calculateOpticalFlowTrajectory fills the caller's Vec4d image and
    trajectory list like the reference (node.cpp:94-99 hands rgb8 frames)."""
    w, h, n = 320, 240, 5
    frames = sequence(mdx, oracle, w, h, n, seed=9, channels=3)
    ofc = mdx.OpticalFlowCalculator(0, w, h)
    try:
        vec_img = np.zeros((h, w, 4))
        trajs = []
        num = ofc.calculateOpticalFlowTrajectory(frames, vec_img, trajs, 10, None, 1.0)
    finally:
        ofc.close()
    ref = oracle.flow_trajectory(frames, pixel_step=10)
    assert num == ref["num_vectors"]
    assert len(trajs) == len(ref["trajectories"])
    for a, b in zip(trajs, ref["trajectories"]):
        np.testing.assert_array_equal(a, b)
    exp = np.zeros((h, w, 4))
    ix = ref["start_pts"].astype(np.int64)
    for i in range(len(ix)):
        exp[ix[i, 1], ix[i, 0]] = ref["vectors"][i]
    np.testing.assert_array_equal(vec_img, exp)


@pytest.mark.gpu
def test_trajectory_flat_and_two_frames(mdx, ctx, oracle):
    frames = [np.full((120, 160), 50, np.uint8), np.full((120, 160), 50, np.uint8)]
    res = ctx.flow_trajectory(frames)
    ref = oracle.flow_trajectory(frames, pixel_step=10)
    _compare(res, ref, "flat")
    assert res.num_vectors == 0


@pytest.mark.gpu
def test_trajectory_chain_equals_per_pass_launches(mdx, oracle, monkeypatch):
    """The chained launch (all passes in one k_lk launch, per-point hand-off) and the per-pass
    launches (MDX_TRAJ_CHAIN=0, read at context creation) give the same bits."""
    w, h, n = 480, 360, 6
    frames = sequence(mdx, oracle, w, h, n, seed=12, channels=3)
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("MDX_TRAJ_CHAIN", mode)
        c = mdx.Context(0, w, h, 1)
        try:
            out[mode] = c.flow_trajectory(frames)
        finally:
            c.close()
    a, b = out["1"], out["0"]
    assert a.num_vectors == b.num_vectors
    np.testing.assert_array_equal(a.traj_len, b.traj_len)
    np.testing.assert_array_equal(a.traj.view(np.uint32), b.traj.view(np.uint32))
    np.testing.assert_array_equal(a.start_pts.view(np.uint32), b.start_pts.view(np.uint32))
    np.testing.assert_array_equal(a.vectors.view(np.uint64), b.vectors.view(np.uint64))
