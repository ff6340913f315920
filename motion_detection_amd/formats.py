"""On-disk formats of the reference for offline parity.

* write_flow: OpticalFlowCalculator::writeFlow (common/src/optical_flow_calculator.cpp:509-541).
  Two text grids, ``<filename>_h`` (dx) and ``<filename>_f`` (dy): one line per grid row
  y = 0, ps, 2ps, ... (< rows), one ", "-separated entry per grid column x = 0, ps, ...; a lost
  point (Vec4d x == -1) writes 0.
* write_trajectories: OpticalFlowCalculator::writeTrajectories (:543-561).  One line per
  trajectory: "x0, y0, x1, y1, ...".
* MotionLogger (common/src/motion_logger.cpp:12-47): writeContour ("frame, id, x, y, x, y, ...")
  and writeBoundingBox ("frame, id, tl.x, tl.y, br.x, br.y"), one line each.

Numbers are formatted like a default std::ostream (precision 6, %g), integers in decimal, so the
files are byte-identical to the reference's (tests/test_formats.py compiles the same loops with
g++/libstdc++ and compares).
"""
from __future__ import annotations

import numpy as np


def _g(v) -> str:
    """operator<<(double) with the default floatfield and precision 6."""
    return "%g" % float(v)


def write_flow(optical_flow_vectors: np.ndarray, filename: str, pixel_step: int,
               entries: np.ndarray | None = None) -> None:
    """optical_flow_vectors: (rows, cols, 4) Vec4d image, as filled by calculateOpticalFlow
    (the grid entries are the only ones read)."""
    v = np.asarray(optical_flow_vectors, dtype=np.float64)
    rows, cols = v.shape[:2]
    with open(filename + "_h", "w") as hf, open(filename + "_f", "w") as vf:
        for i in range(0, rows, pixel_step):
            hs, vs = [], []
            for j in range(0, cols, pixel_step):
                e = v[i, j]
                if e[0] == -1.0:
                    hs.append(_g(0.0)); vs.append(_g(0.0))
                else:
                    hs.append(_g(e[2])); vs.append(_g(e[3]))
            hf.write(", ".join(hs) + "\n")
            vf.write(", ".join(vs) + "\n")


def write_trajectories(trajectories, filename: str) -> None:
    with open(filename, "w") as tf:
        for traj in trajectories:
            t = np.asarray(traj, dtype=np.float32)
            tf.write(", ".join(f"{_g(p[0])}, {_g(p[1])}" for p in t) + "\n")


class MotionLogger:
    def __init__(self, log_filepath: str | None = None):
        self._f = open(log_filepath, "w") if log_filepath else None

    def setFileName(self, log_filepath: str):
        if self._f:
            self._f.close()
        self._f = open(log_filepath, "w")

    def writeContour(self, points, frame_number: int, contour_id: int):
        s = f"{int(frame_number)}, {int(contour_id)}"
        for p in points:
            s += f", {int(p[0])}, {int(p[1])}"
        self._f.write(s + "\n")

    def writeBoundingBox(self, rect, frame_number: int, contour_id: int):
        """rect = (x, y, width, height) like cv::Rect; br() = (x + width, y + height)."""
        x, y, wd, ht = (int(r) for r in rect)
        self._f.write(f"{int(frame_number)}, {int(contour_id)}, {x}, {y}, {x + wd}, {y + ht}\n")

    def close(self):
        if self._f:
            self._f.close()
            self._f = None

    def __del__(self):
        self.close()
