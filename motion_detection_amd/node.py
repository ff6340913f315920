"""ROS-free core of MotionDetectionNode for the hot path (the drop-in boundary's caller).

Reproduces the ingest semantics of MotionDetectionNode::imageCallback
(ros/src/motion_detection_node.cpp:235-287) and the runOpticalFlow caller (:76-92), without
ROS: frames arrive as ``Image`` records shaped like sensor_msgs/Image (height, width,
encoding, step, data).  Parameters mirror the node's ROS params (:29-44, :237-245):

* skip_frames (default 1) and num_motions (default 2) are re-read on every frame;
  trajectory_size = 2*num_motions + 1, or 2 when egomotion is false (:241-245).
* a frame is dropped unless global_frame_count % skip_frames == 0 (:247).  The counter
  advances on every call: on a dropped frame at :247, on a kept one at :454 (:315 when no
  trajectory survives), so skip_frames = k keeps frames 0, k, 2k, ...
* raw frames go into a ring of trajectory_size (:248-261); once full, the last two
  frames are converted to rgb8 (cv_bridge toCvCopy, :271) and handed to the calculator.

Publishing is a callback: ``on_result(result)`` receives the FlowResult (vectors + mask),
standing in for publishImage on ~optical_flow_image (:83-85).

By default (``live_chain=True``, as the reference's imageCallback and host/mdx_host.h) the callback
follows the reference's live branch (:266-348): every ring frame goes to
calculateOpticalFlowTrajectory (:295, runOpticalFlowTrajectory :94-110); with egomotion and at
least one complete trajectory, fitSubspace(trajectories, outlier_points, num_motions, sigma) follows
(:341-348).  ``on_result`` then receives a LiveResult.  ``live_chain=False`` drives the pair path
the north star names (runOpticalFlow, :76-92) on the ring's last two frames, the only one that
produces the motion mask.
"""
from __future__ import annotations

from collections import deque
from dataclasses import dataclass
from typing import Callable

import numpy as np

from . import _lib
from .optical_flow_calculator import OpticalFlowCalculator

ENCODINGS = {"mono8": (1, _lib.FMT_GRAY8), "rgb8": (3, _lib.FMT_RGB8), "bgr8": (3, _lib.FMT_BGR8)}


@dataclass
class Image:
    """Minimal sensor_msgs/Image."""
    height: int
    width: int
    encoding: str
    step: int
    data: bytes | np.ndarray

    @staticmethod
    def from_array(a: np.ndarray, encoding: str | None = None) -> "Image":
        a = np.ascontiguousarray(a, dtype=np.uint8)
        enc = encoding or ("mono8" if a.ndim == 2 else "rgb8")
        return Image(a.shape[0], a.shape[1], enc, a.strides[0], a.tobytes())


def to_rgb8(msg: Image) -> np.ndarray:
    """cv_bridge::toCvCopy(msg, "rgb8"): mono8 is replicated, bgr8 is reordered."""
    if msg.encoding not in ENCODINGS:
        raise ValueError(f"unsupported encoding {msg.encoding!r}")
    cn, _ = ENCODINGS[msg.encoding]
    buf = np.frombuffer(bytes(msg.data) if not isinstance(msg.data, np.ndarray) else msg.data.tobytes(), np.uint8)
    rows = buf[: msg.step * msg.height].reshape(msg.height, msg.step)[:, : msg.width * cn]
    if cn == 1:
        return np.repeat(rows[:, :, None], 3, axis=2)
    px = rows.reshape(msg.height, msg.width, 3)
    return px[:, :, ::-1].copy() if msg.encoding == "bgr8" else px.copy()


@dataclass
class LiveResult:
    """Outputs of the live branch (node.cpp:266-348) up to the clustering it hands them to."""
    num_vectors: int
    optical_flow_vectors: np.ndarray     # (h, w, 4) Vec4d image (runOpticalFlowTrajectory :97-99)
    trajectories: list                   # complete trajectories, (T, 2) each
    outlier_points: list                 # fitSubspace's (egomotion only)
    subspace: list                       # fitSubspace's return value (egomotion only)


class MotionDetectionNode:
    def __init__(self, params: dict | None = None, on_result: Callable | None = None, device: int = 0):
        # the reference's defaults (node.cpp:29-44, :237-240, :346); egomotion true (:40) sets a
        # ring of 2*num_motions+1 frames, and imageCallback always runs the live branch on it
        # (live_chain True; False selects the pair path on the ring's last two frames)
        self.params = {"pixel_step": 10, "min_vector_size": 1.0, "skip_frames": 1, "num_motions": 2,
                       "egomotion": True, "use_all_frames": True, "sigma": 0.5, "live_chain": True}
        if params:
            self.params.update(params)
        self.on_result = on_result
        self.raw_images: deque = deque()
        self.global_frame_count = 0
        self.image_received = False
        self.frames_processed = 0
        self.ofc = OpticalFlowCalculator(device=device)
        self.od = None                                    # OutlierDetector, created on first use
        self._device = device

    @property
    def trajectory_size(self) -> int:
        # node.cpp:241-245
        return 2 if not self.params["egomotion"] else 2 * int(self.params["num_motions"]) + 1

    def image_callback(self, msg: Image):
        skip = int(self.params.get("skip_frames", 1))
        if self.global_frame_count % skip != 0:          # :247
            self.global_frame_count += 1
            return None
        ts = self.trajectory_size
        if len(self.raw_images) < ts:                     # :248-261
            self.raw_images.append(msg)
            if len(self.raw_images) == ts:
                self.image_received = True
        else:
            self.raw_images.append(msg)
            self.raw_images.popleft()
            self.image_received = True
        out = None
        if self.params.get("use_all_frames", True) and self.image_received:
            if self.params.get("live_chain", True):
                out = self.run_live_chain([to_rgb8(m) for m in self.raw_images])   # :266-295
            else:
                frames = [to_rgb8(m) for m in list(self.raw_images)[-2:]]   # :266-287
                out = self.run_optical_flow(frames[0], frames[1])
        self.global_frame_count += 1                          # :454
        return out

    def run_live_chain(self, images: list):
        """runOpticalFlowTrajectory (node.cpp:94-110) then, with egomotion, fitSubspace (:341-348)."""
        h, w = images[0].shape[:2]
        vec = np.zeros((h, w, 4))                         # cv::Mat::zeros(rows, cols, CV_32FC4) (:97)
        trajectories: list = []
        num = self.ofc.calculateOpticalFlowTrajectory(images, vec, trajectories, int(self.params["pixel_step"]),
                                                      None, float(self.params["min_vector_size"]))
        outliers: list = []
        subspace: list = []
        if trajectories and self.params["egomotion"]:
            if self.od is None:
                from .outlier_detector import OutlierDetector
                self.od = OutlierDetector(seed=self.params.get("seed"), device=self._device)
            subspace = self.od.fitSubspace(trajectories, outliers, int(self.params["num_motions"]),
                                           float(self.params["sigma"]))
        self.frames_processed += 1
        res = LiveResult(num, vec, trajectories, outliers, subspace)
        if self.on_result is not None:
            self.on_result(res)
        return res

    def run_optical_flow(self, image1: np.ndarray, image2: np.ndarray):
        """runOpticalFlow (node.cpp:76-92)."""
        res = self.ofc.compute(image1, image2, int(self.params["pixel_step"]), float(self.params["min_vector_size"]),
                               fmt=_lib.FMT_RGB8)
        self.frames_processed += 1
        if self.on_result is not None:
            self.on_result(res)
        return res
