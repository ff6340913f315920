"""Mirror of the reference's OpticalFlowCalculator interface for the hot path.

Reference: class OpticalFlowCalculator (common/include/motion_detection/optical_flow_calculator.h:13-33),
method calculateOpticalFlow (common/src/optical_flow_calculator.cpp:30-130).  Same name,
argument meaning and return value; the output Mats become numpy arrays filled in place:

    num_vectors = ofc.calculateOpticalFlow(image1, image2, optical_flow_vectors,
                                           pixel_step, comp, min_vector_size)

* image1/image2: (h, w, 3) rgb8 (what the node hands over, node.cpp:271) or (h, w) mono8.
* optical_flow_vectors: (h, w, 4) float64, zero-initialised by the caller like
  cv::Mat::zeros(rows, cols, CV_32FC4) (node.cpp:81).  Entry [y, x] of every grid point
  receives the reference's Vec4d: (x, y, dx, dy) for an accepted vector, (x, y, 0, 0) for a
  tracked point below min_vector_size, (-1, -1, 0, 0) for a lost point (:78-117).  The
  reference stores Vec4d into a CV_32FC4 Mat (16-B elements), which aliases neighbouring
  grid entries in memory; the mirror keeps one entry per grid point (semantic parity).
* comp: (h, w) uint8; receives the thresholded frame difference when num_vectors > 0
  (:118-128).  With 1..3 vectors the reference reads past src_points (UB); here comp is
  zero-filled instead.

calculateOpticalFlowTrajectory (:133-257), the node's live caller (node.cpp:94-110), has the
same form:

    num_vectors = ofc.calculateOpticalFlowTrajectory(images, optical_flow_vectors, trajectories,
                                                     pixel_step, comp, min_vector_size)

* images: list of >= 2 frames (rgb8 or mono8).
* optical_flow_vectors: (h, w, 4) float64; the last pass's Vec4d of every point is stored at
  [(int)y, (int)x] of the point entering that pass, in point order (later points overwrite
  earlier ones at the same pixel, as the reference's stores do).
* trajectories: a list, extended with the complete trajectories ((nimg, 2) float32 arrays).
* comp is not touched (the reference never writes it here).

All arithmetic runs on the MI355X through libmdx.so; there is no CPU fallback.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .context import Context, FlowResult, grid_points


class OpticalFlowCalculator:
    """Stateless like the reference (optical_flow_calculator.cpp:20-28), except for the
    device context it keeps so the per-frame path does not reallocate."""

    def __init__(self, device: int = 0, max_w: int = 1920, max_h: int = 1080):
        self._device = device
        self._ctx: Context | None = None
        self._cap = (max_w, max_h)

    def _context(self, w: int, h: int, pixel_step: int, min_vector_size: float) -> Context:
        if self._ctx is None or w > self._cap[0] or h > self._cap[1]:
            self._cap = (max(self._cap[0], w), max(self._cap[1], h))
            if self._ctx is not None:
                self._ctx.close()
            self._ctx = Context(self._device, self._cap[0], self._cap[1], 1)
        self._ctx.set_params(pixel_step=int(pixel_step), min_vector_size=float(min_vector_size))
        return self._ctx

    def calculateOpticalFlow(self, image1: np.ndarray, image2: np.ndarray, optical_flow_vectors: np.ndarray,
                             pixel_step: int, comp: np.ndarray | None, min_vector_size: float) -> int:
        image1 = np.asarray(image1)
        image2 = np.asarray(image2)
        h, w = image1.shape[:2]
        fmt = _lib.FMT_GRAY8 if image1.ndim == 2 else _lib.FMT_RGB8
        res = self.compute(image1, image2, pixel_step, min_vector_size, fmt=fmt, want_mask=comp is not None)
        if optical_flow_vectors is not None:
            if optical_flow_vectors.shape[:2] != (h, w) or optical_flow_vectors.shape[-1] != 4:
                raise ValueError("optical_flow_vectors must be (h, w, 4)")
            pts = grid_points(w, h, pixel_step).astype(np.int64)
            optical_flow_vectors[pts[:, 1], pts[:, 0], :] = res.vectors
        if comp is not None and res.num_vectors > 0:
            comp[...] = res.mask
        return res.num_vectors

    def calculateOpticalFlowTrajectory(self, images, optical_flow_vectors: np.ndarray | None, trajectories: list,
                                       pixel_step: int, comp: np.ndarray | None, min_vector_size: float) -> int:
        imgs = [np.asarray(im) for im in images]
        h, w = imgs[0].shape[:2]
        fmt = _lib.FMT_GRAY8 if imgs[0].ndim == 2 else _lib.FMT_RGB8
        ctx = self._context(w, h, pixel_step, min_vector_size)
        res = ctx.flow_trajectory(imgs, fmt=fmt)
        if optical_flow_vectors is not None:
            if optical_flow_vectors.shape[:2] != (h, w) or optical_flow_vectors.shape[-1] != 4:
                raise ValueError("optical_flow_vectors must be (h, w, 4)")
            ix = res.start_pts.astype(np.int64)   # (int) truncation of the float position
            ok = (ix[:, 0] >= 0) & (ix[:, 0] < w) & (ix[:, 1] >= 0) & (ix[:, 1] < h)
            for i in np.nonzero(ok)[0]:           # point order: last store wins
                optical_flow_vectors[ix[i, 1], ix[i, 0], :] = res.vectors[i]
        trajectories.extend(res.trajectories)
        return res.num_vectors

    def compute(self, image1: np.ndarray, image2: np.ndarray, pixel_step: int = 10, min_vector_size: float = 1.0,
                fmt: int | None = None, want_mask: bool = True) -> FlowResult:
        """Pythonic form: every output of the path in one FlowResult."""
        h, w = np.asarray(image1).shape[:2]
        ctx = self._context(w, h, pixel_step, min_vector_size)
        return ctx.flow_warp_diff(image1, image2, fmt=fmt, want_mask=want_mask)

    def close(self):
        if self._ctx is not None:
            self._ctx.close()
            self._ctx = None
