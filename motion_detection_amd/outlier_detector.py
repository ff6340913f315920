"""Mirror of the reference's OutlierDetector::fitSubspace for the trajectory path.

Reference: class OutlierDetector (common/include/motion_detection/outlier_detector.h:14-40),
constructor (common/src/outlier_detector.cpp:15-31: srand(time(NULL)) and the chi-square table),
fitSubspace (:236-331), called by the node on the complete trajectories
(ros/src/motion_detection_node.cpp:345-348):

    od = OutlierDetector()                     # seed=None: time(NULL), as the reference
    subspace = od.fitSubspace(trajectories, outlier_points, num_motions, sigma)

* trajectories: list of (T, 2) arrays (OpticalFlowCalculator.calculateOpticalFlowTrajectory's).
* outlier_points: a list, extended with each outlier trajectory's second-to-last point (:322).
* returns the winning sample's trajectories (4*num_motions of them, repeats possible; empty when
  no hypothesis found an inlier), like the reference's return value.

The generator is glibc's rand() restated (mdx_srand / mdx_rand), one stream per detector across
calls, like the reference's.  All arithmetic runs on the MI355X through libmdx.so.
"""
from __future__ import annotations

import ctypes as C
import time

import numpy as np

from . import _lib
from .context import Context, SubspaceResult


class OutlierDetector:
    def __init__(self, seed: int | None = None, device: int = 0, precision: int = _lib.SUBSPACE_F64):
        """precision: SUBSPACE_F64 (default, stable) or SUBSPACE_F32 (the reference's float
        arithmetic shape; see include/mdx.h mdx_fit_subspace)."""
        self.precision = int(precision)
        self.rng = _lib.MdxRandState()
        self.seed = int(time.time()) & 0xFFFFFFFF if seed is None else int(seed) & 0xFFFFFFFF
        _lib.lib().mdx_srand(C.byref(self.rng), self.seed)
        self._device = device
        self._ctx: Context | None = None
        self.last: SubspaceResult | None = None

    def fitSubspace(self, trajectories, outlier_points: list, num_motions: int, sigma: float) -> list:
        traj = np.ascontiguousarray(np.asarray(trajectories, dtype=np.float32))
        if self._ctx is None:
            self._ctx = Context(self._device, 64, 64, 1, subspace_precision=self.precision)
        res = self._ctx.fit_subspace(traj, num_motions, sigma, self.rng)
        self.last = res
        outlier_points.extend(tuple(p) for p in res.outlier_points)
        return [traj[i] for i in res.columns if i >= 0]

    def close(self):
        if self._ctx is not None:
            self._ctx.close()
            self._ctx = None
