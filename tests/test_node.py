"""Host-side mirror of the reference interface, on CPU.

* MotionDetectionNode ingest (reference ros/src/motion_detection_node.cpp:235-287, runOpticalFlow
  :76-92) with a recording stand-in for the calculator: frame ring, skip_frames quirk, rgb8
  conversion (cv_bridge toCvCopy, :271).
* OpticalFlowCalculator.calculateOpticalFlow's output placement (optical_flow_calculator.cpp:78-128):
  the Vec4d per grid point and comp, with the device compute replaced by a stub that returns the
  oracle's result (the GPU path itself is exercised by tests/test_parity_gpu.py).
"""
import numpy as np
import pytest

import motion_detection_amd as m
from motion_detection_amd.context import FlowResult, grid_points
from motion_detection_amd.node import Image, MotionDetectionNode, to_rgb8


class RecordingCalc:
    def __init__(self):
        self.calls = []

    def compute(self, image1, image2, pixel_step, min_vector_size, fmt=None, want_mask=True):
        self.calls.append((image1.copy(), image2.copy(), pixel_step, min_vector_size, fmt))
        return len(self.calls)


def frame(v, h=6, w=8, enc="mono8"):
    a = np.full((h, w) if enc == "mono8" else (h, w, 3), v, np.uint8)
    if enc != "mono8":
        a[..., 0] = v
        a[..., 1] = v + 1
        a[..., 2] = v + 2
    return Image.from_array(a, enc)


def make_node(**params):
    params.setdefault("live_chain", False)   # these tests drive the pair path (runOpticalFlow)
    n = MotionDetectionNode(params)       # no device work at construction
    n.ofc = RecordingCalc()
    return n


def test_to_rgb8_conversions():
    g = np.arange(12, dtype=np.uint8).reshape(3, 4)
    assert np.array_equal(to_rgb8(Image.from_array(g, "mono8")), np.repeat(g[..., None], 3, 2))
    rgb = np.arange(36, dtype=np.uint8).reshape(3, 4, 3)
    assert np.array_equal(to_rgb8(Image.from_array(rgb, "rgb8")), rgb)
    assert np.array_equal(to_rgb8(Image.from_array(rgb, "bgr8")), rgb[..., ::-1])
    # row padding (step > width*channels) is dropped
    padded = np.zeros((3, 6), np.uint8)
    padded[:, :4] = g
    msg = Image(3, 4, "mono8", 6, padded.tobytes())
    assert np.array_equal(to_rgb8(msg)[..., 0], g)
    with pytest.raises(ValueError):
        to_rgb8(Image(1, 1, "yuv422", 2, b"\0\0"))


def test_pairs_of_consecutive_frames():
    n = make_node(egomotion=False)
    assert n.trajectory_size == 2
    assert n.image_callback(frame(10)) is None            # ring not yet full
    assert n.image_callback(frame(20)) == 1
    assert n.image_callback(frame(30)) == 2
    (a1, b1, ps, mvs, fmt), (a2, b2, *_) = n.ofc.calls
    assert a1[0, 0, 0] == 10 and b1[0, 0, 0] == 20 and a2[0, 0, 0] == 20 and b2[0, 0, 0] == 30
    assert a1.shape == (6, 8, 3) and fmt == m.FMT_RGB8      # cv_bridge rgb8 copy (node.cpp:271)
    assert (ps, mvs) == (10, 1.0)
    assert n.frames_processed == 2


def test_reference_defaults():
    n = MotionDetectionNode()
    assert n.params["egomotion"] is True                     # node.cpp:40
    assert n.params["live_chain"] is True                    # imageCallback's live branch (:266-348)
    assert n.trajectory_size == 5                            # 2*num_motions + 1 (:241)


def test_default_first_result_is_the_live_branch_on_frame_4():
    """Under the defaults the ring fills to 2*num_motions+1 = 5 frames and the fifth callback runs
    the live branch on all five (node.cpp:241-295), as the reference and host/mdx_host.h do."""
    n = MotionDetectionNode()
    rec = RecordingLive()
    n.ofc = rec
    n.od = rec
    out = [n.image_callback(frame(v)) for v in range(6)]
    assert [i for i, o in enumerate(out) if o is not None] == [4, 5]
    assert [im[0, 0, 0] for im in rec.traj_calls[0][0]] == [0, 1, 2, 3, 4]
    assert [im[0, 0, 0] for im in rec.traj_calls[1][0]] == [1, 2, 3, 4, 5]
    assert len(rec.fit_calls) == 2


def test_egomotion_ring_size():
    n = make_node(egomotion=True, num_motions=2)
    assert n.trajectory_size == 5                           # 2*num_motions + 1 (node.cpp:241-245)
    for v in range(4):
        assert n.image_callback(frame(v)) is None
    assert n.image_callback(frame(4)) == 1
    a, b, *_ = n.ofc.calls[0]
    assert a[0, 0, 0] == 3 and b[0, 0, 0] == 4              # the last two frames of the ring


def test_skip_frames():
    # node.cpp:247 drops a frame unless the counter is a multiple of skip_frames; the counter
    # advances on every call (:247 dropped, :454 kept), so frames 0, 3, 6, ... are kept
    n = make_node(skip_frames=3, egomotion=False)
    out = [n.image_callback(frame(v)) for v in range(10)]
    assert n.global_frame_count == 10
    assert [i for i, o in enumerate(out) if o is not None] == [3, 6, 9]   # pairs (0,3), (3,6), (6,9)
    assert [(c[0][0, 0, 0], c[1][0, 0, 0]) for c in n.ofc.calls] == [(0, 3), (3, 6), (6, 9)]


def test_use_all_frames_false_never_runs():
    n = make_node(use_all_frames=False)
    for v in range(4):
        assert n.image_callback(frame(v)) is None
    assert not n.ofc.calls


# ---------------------------------------------------------------- calculateOpticalFlow placement

class OracleStubCalc(m.OpticalFlowCalculator):
    """calculateOpticalFlow's host logic over the oracle's result (CPU only)."""

    def compute(self, image1, image2, pixel_step=10, min_vector_size=1.0, fmt=None, want_mask=True):
        from oracle import pyoracle
        r = pyoracle.calculate_optical_flow(image1, image2, pixel_step=pixel_step, min_vector_size=min_vector_size,
                                            want_mask=want_mask)
        code = m.MDX_OK if r["num_vectors"] >= 4 or r["num_vectors"] == 0 else m.MDX_EDEGENERATE
        mask = r["mask"]
        if mask is not None and 0 < r["num_vectors"] < 4:
            mask = np.zeros_like(mask)
        return FlowResult(r["num_vectors"], r["next_pts"], r["status"], r["vectors"], mask, r["H"], code)


def test_calculate_optical_flow_fills_reference_outputs(oracle):
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "synth_160x120_rgb.npz"))
    ps, mvs = int(g["pixel_step"]), float(g["min_vector_size"])
    calc = OracleStubCalc()
    vec = np.zeros((120, 160, 4), np.float64)           # cv::Mat::zeros(rows, cols, CV_32FC4) (node.cpp:81)
    comp = np.zeros((120, 160), np.uint8)
    num = calc.calculateOpticalFlow(g["img1"], g["img2"], vec, ps, comp, mvs)
    assert num == int(g["num_vectors"])
    pts = grid_points(160, 120, ps).astype(int)
    assert np.array_equal(vec[pts[:, 1], pts[:, 0]], g["vectors"])
    off_grid = np.ones((120, 160), bool)
    off_grid[pts[:, 1], pts[:, 0]] = False
    assert np.all(vec[off_grid] == 0)
    assert np.array_equal(comp, g["mask"])
    with pytest.raises(ValueError):
        calc.calculateOpticalFlow(g["img1"], g["img2"], np.zeros((10, 10, 4)), ps, comp, mvs)


def test_calculate_optical_flow_no_vectors_leaves_comp(oracle):
    f = np.full((48, 64), 50, np.uint8)
    comp = np.full((48, 64), 7, np.uint8)
    vec = np.zeros((48, 64, 4))
    assert OracleStubCalc().calculateOpticalFlow(f, f, vec, 8, comp, 1.0) == 0
    assert np.all(comp == 7)                              # :118 no mask branch: comp untouched
    pts = grid_points(64, 48, 8).astype(int)
    assert np.all(vec[pts[:, 1], pts[:, 0], :2] == -1)


class RecordingLive:
    """Stand-ins for the trajectory calculator and the detector (GPU work is tested elsewhere)."""
    def __init__(self):
        self.traj_calls, self.fit_calls = [], []

    def calculateOpticalFlowTrajectory(self, images, vec, trajectories, pixel_step, comp, mvs):
        self.traj_calls.append(([im.copy() for im in images], pixel_step, mvs))
        trajectories.extend([np.zeros((len(images), 2), np.float32)] * 3)
        return 7

    def fitSubspace(self, trajectories, outlier_points, num_motions, sigma):
        self.fit_calls.append((len(trajectories), num_motions, sigma))
        outlier_points.append((1.0, 2.0))
        return trajectories[:1]


def test_live_chain_trajectory_and_subspace():
    """Live branch (node.cpp:266-348): all ring frames to the trajectory call; with egomotion,
    fitSubspace on its complete trajectories with num_motions and sigma."""
    n = MotionDetectionNode({"egomotion": True, "num_motions": 2, "sigma": 0.7, "live_chain": True})
    rec = RecordingLive()
    n.ofc = rec
    n.od = rec
    for v in range(4):
        assert n.image_callback(frame(v)) is None
    res = n.image_callback(frame(4))
    imgs, ps, mvs = rec.traj_calls[0]
    assert [im[0, 0, 0] for im in imgs] == [0, 1, 2, 3, 4] and imgs[0].shape == (6, 8, 3)
    assert (ps, mvs) == (10, 1.0)
    assert rec.fit_calls == [(3, 2, 0.7)]
    assert res.num_vectors == 7 and res.outlier_points == [(1.0, 2.0)] and len(res.subspace) == 1
    # without egomotion: trajectories only (the reference clusters them instead, out of scope)
    n2 = MotionDetectionNode({"live_chain": True, "egomotion": False})
    rec2 = RecordingLive()
    n2.ofc = rec2
    n2.od = rec2
    n2.image_callback(frame(1))
    r2 = n2.image_callback(frame(2))
    assert len(rec2.traj_calls[0][0]) == 2 and rec2.fit_calls == [] and r2.outlier_points == []
