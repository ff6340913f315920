"""On-disk formats: writeFlow / writeTrajectories
(common/src/optical_flow_calculator.cpp:509-561) and MotionLogger (common/src/motion_logger.cpp:37-47).

The expected bytes come from a small C++ program (written here, compiled with this machine's g++)
that runs the reference's own output loops with std::ofstream on the same values, so the number
formatting is libstdc++'s.  Values include the lost-point rule (x == -1 -> 0), negative zero,
large/small magnitudes and float32 trajectory coordinates.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

from motion_detection_amd.formats import MotionLogger, write_flow, write_trajectories

CPP = r"""
#include <fstream>
#include <cstdio>
#include <string>
#include <vector>
int main(int argc, char** argv) {
    // args: rows cols ps, then rows*cols*4 doubles on stdin; trajectories: n T then floats
    int rows, cols, ps;
    if (std::scanf("%d %d %d", &rows, &cols, &ps) != 3) return 1;
    std::vector<double> v((size_t)rows * cols * 4);
    for (auto& x : v) if (std::scanf("%lf", &x) != 1) return 1;
    std::string f = argv[1];
    std::ofstream hfile(f + "_h"), vfile(f + "_f");
    for (int i = 0; i < rows; i = i + ps) {
        for (int j = 0; j < cols; j = j + ps) {
            if (j != 0) { hfile << ", "; vfile << ", "; }
            const double* e = &v[((size_t)i * cols + j) * 4];
            if (e[0] == -1.0) { hfile << 0.0; vfile << 0.0; }
            else { hfile << e[2]; vfile << e[3]; }
        }
        hfile << std::endl; vfile << std::endl;
    }
    int n, T;
    if (std::scanf("%d %d", &n, &T) != 2) return 1;
    std::ofstream tfile(f + "_traj");
    for (int i = 0; i < n; i++) {
        for (int j = 0; j < T; j++) {
            float x, y;
            if (std::scanf("%f %f", &x, &y) != 2) return 1;
            if (j != 0) tfile << ", ";
            tfile << x << ", " << y;
        }
        tfile << std::endl;
    }
    std::ofstream lfile(f + "_log");
    lfile << 12 << ", " << 3 << ", " << 10 << ", " << 20 << ", " << 40 << ", " << 70 << std::endl;   // writeBoundingBox
    lfile << 13 << ", " << 0;
    int pts[3][2] = {{1, 2}, {3, 4}, {-5, 6}};
    for (auto& p : pts) lfile << ", " << p[0] << ", " << p[1];                                     // writeContour
    lfile << std::endl;
    return 0;
}
"""


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++ for the libstdc++ reference bytes")
def test_formats_match_libstdcxx(tmp_path):
    rng = np.random.default_rng(4)
    rows, cols, ps = 23, 31, 5
    v = np.zeros((rows, cols, 4))
    v[..., 0] = rng.integers(-1, 3, (rows, cols)).astype(float)        # some lost points (x == -1)
    v[..., 2] = rng.normal(0, 3, (rows, cols)) * 10.0 ** rng.integers(-7, 8, (rows, cols))
    v[..., 3] = rng.normal(0, 1, (rows, cols)).astype(np.float32)
    v[0, 5, 0] = 0.0; v[0, 5, 2] = -0.0                                 # negative zero
    v[5, 0, 2] = 123456789.0; v[5, 5, 3] = 1e-300
    traj = (rng.normal(300, 100, (7, 5, 2))).astype(np.float32)
    traj[0, 0] = (0.1, 1234567.0)

    exe = tmp_path / "fmt"
    src = tmp_path / "fmt.cpp"
    src.write_text(CPP)
    subprocess.run(["g++", "-O1", "-o", str(exe), str(src)], check=True)
    inp = f"{rows} {cols} {ps}\n" + " ".join(repr(float(x)) for x in v.ravel()) + "\n"
    inp += f"{traj.shape[0]} {traj.shape[1]}\n" + " ".join(repr(float(x)) for x in traj.ravel()) + "\n"
    ref = str(tmp_path / "ref")
    subprocess.run([str(exe), ref], input=inp.encode(), check=True)

    ours = str(tmp_path / "ours")
    write_flow(v, ours, ps)
    write_trajectories(list(traj), ours + "_traj")
    lg = MotionLogger(ours + "_log")
    lg.writeBoundingBox((10, 20, 30, 50), 12, 3)
    lg.writeContour([(1, 2), (3, 4), (-5, 6)], 13, 0)
    lg.close()
    for suffix in ("_h", "_f", "_traj", "_log"):
        a, b = open(ours + suffix, "rb").read(), open(ref + suffix, "rb").read()
        assert a == b, f"{suffix}: {a[:200]!r} vs {b[:200]!r}"
    assert os.path.getsize(ours + "_h") > 0
