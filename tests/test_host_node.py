"""The compiled C++ caller of the boundary (host/: mdx_host.cpp + mdx_node), no Python between the
frame bytes and the C-ABI.

Reference: MotionDetectionNode (ros/src/motion_detection_node.cpp) -- imageCallback's ring, skip
and rgb8 semantics (:235-287), runOpticalFlow (:76-92), runOpticalFlowTrajectory + fitSubspace
(:94-110, :341-348), publishImage's RGB8 messages (:217-223), writeFlow / writeTrajectories
(common/src/optical_flow_calculator.cpp:509-562) and MotionLogger's format (common/src/motion_logger.cpp:31-47).

The tests write a recorded stream of sensor_msgs/Image-shaped frames to a file; the g++-built
binary reads it, runs the node through libmdx.so and writes every published image and output.
The checker is the oracle (oracle/) replaying the reference's semantics on the same frames:
next_pts (float32 bits), status, mask, H, num_vectors, trajectories, subspace outliers and the
on-disk files must be identical (the files through motion_detection_amd.formats, itself
byte-checked against libstdc++ in test_formats.py).
"""
import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "host")
EXE = os.path.join(HOST, "mdx_node")


@pytest.fixture(scope="module")
def node_exe(mdx):
    if shutil.which("g++") is None:
        pytest.skip("needs g++")
    subprocess.run(["make", "-s", "-C", HOST], check=True)
    return EXE


def write_frames(path, frames):
    """frames: list of (array, encoding); the binary's MDXF stream of sensor_msgs/Image records."""
    with open(path, "wb") as f:
        f.write(b"MDXF" + struct.pack("<I", len(frames)))
        for a, enc in frames:
            a = np.ascontiguousarray(a, np.uint8)
            h, w = a.shape[:2]
            step = a.strides[0]
            f.write(struct.pack("<4I", h, w, step, len(enc)) + enc.encode() + a.tobytes())


def run_node(exe, tmp_path, frames, **params):
    fpath = tmp_path / "frames.bin"
    write_frames(str(fpath), frames)
    out = tmp_path / "out"
    out.mkdir()
    args = [exe, str(fpath), str(out)] + [f"{k}={int(v) if isinstance(v, bool) else v}" for k, v in params.items()]
    p = subprocess.run(args, capture_output=True, text=True, timeout=300)
    return p, out


def to_rgb8(a, enc):
    if enc == "mono8":
        return np.repeat(a[:, :, None], 3, axis=2)
    return a[:, :, ::-1].copy() if enc == "bgr8" else a.copy()


def kept_frames(n, skip):
    """imageCallback's skip rule (:247, :454): the counter advances on every call."""
    return [i for i in range(n) if i % skip == 0]


def read_res(path, live, npts=0, w=0, h=0):
    b = open(path, "rb").read()
    num, rc, w, h, npts, ntraj, tl, nout = struct.unpack_from("<8i", b, 0)
    o = 32
    H = np.frombuffer(b, np.float64, 9, o).reshape(3, 3)
    o += 72
    r = dict(num=num, rc=rc, w=w, h=h, npts=npts, H=H)
    if not live:
        r["next_pts"] = np.frombuffer(b, np.float32, 2 * npts, o).reshape(npts, 2)
        o += 8 * npts
        r["status"] = np.frombuffer(b, np.uint8, npts, o)
        o += npts
        r["mask"] = np.frombuffer(b, np.uint8, w * h, o).reshape(h, w)
    else:
        r["traj"] = np.frombuffer(b, np.float32, ntraj * tl * 2, o).reshape(ntraj, tl, 2)
        o += ntraj * tl * 8
        r["outliers"] = np.frombuffer(b, np.float32, nout * 2, o).reshape(nout, 2)
        o += nout * 8
        nc = struct.unpack_from("<i", b, o)[0]
        r["columns"] = np.frombuffer(b, np.int32, nc, o + 4)
    return r


def vector_image(vectors, w, h, ps):
    v = np.zeros((h, w, 4))
    ny = -(-h // ps)
    for k in range(len(vectors)):
        v[(k % ny) * ps, (k // ny) * ps] = vectors[k]
    return v


def test_node_binary_fails_cleanly_without_a_device(node_exe, tmp_path, mdx):
    """CPU: the node binary links libmdx.so and reports the missing GPU as an error, exit 1."""
    a, b, _ = mdx.synth_pair(5, 64, 48, 3)
    env = dict(os.environ, HIP_VISIBLE_DEVICES="-1")
    fpath = tmp_path / "f.bin"
    write_frames(str(fpath), [(a, "rgb8"), (b, "rgb8")])
    p = subprocess.run([node_exe, str(fpath), str(tmp_path), "live_path=0", "egomotion=0"], capture_output=True,
                       text=True, timeout=120, env=env)
    if p.returncode == 0:
        pytest.skip("a GPU is visible here")
    assert p.returncode == 1 and "mdx_create" in p.stderr, p.stderr


CPP_FMT = r"""
#include "mdx_host.h"
#include <cstdio>
#include <vector>
int main(int, char** argv) {
    int rows, cols, ps, n, T;
    if (std::scanf("%d %d %d", &rows, &cols, &ps) != 3) return 1;
    std::vector<double> v((size_t)rows * cols * 4);
    for (auto& x : v) if (std::scanf("%lf", &x) != 1) return 1;
    mdx_host::write_flow(v, cols, rows, ps, argv[1]);
    if (std::scanf("%d %d", &n, &T) != 2) return 1;
    std::vector<std::vector<float>> t(n, std::vector<float>(2 * T));
    for (auto& tr : t) for (auto& x : tr) if (std::scanf("%f", &x) != 1) return 1;
    mdx_host::write_trajectories(t, std::string(argv[1]) + "_traj");
    mdx_host::MotionLogger lg(std::string(argv[1]) + "_log");
    lg.write_bounding_box(10, 20, 30, 50, 12, 3);
    lg.write_contour({1, 2, 3, 4, -5, 6}, 13, 0);
    return 0;
}
"""


def test_host_writers_match_python_formats(tmp_path, mdx):
    """CPU: the C++ host's writeFlow / writeTrajectories / MotionLogger bytes equal formats.py's
    (which test_formats.py pins to the reference's libstdc++ loops)."""
    if shutil.which("g++") is None:
        pytest.skip("needs g++")
    from motion_detection_amd.formats import MotionLogger, write_flow, write_trajectories
    src = tmp_path / "fmt.cpp"
    src.write_text(CPP_FMT)
    exe = tmp_path / "fmt"
    libdir = os.path.join(ROOT, "motion_detection_amd", "lib")
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", HOST, "-I", os.path.join(ROOT, "include"), str(src),
                    os.path.join(HOST, "mdx_host.cpp"), "-L", libdir, "-lmdx", f"-Wl,-rpath,{libdir}", "-o", str(exe)],
                   check=True)
    rng = np.random.default_rng(9)
    rows, cols, ps = 19, 27, 4
    v = np.zeros((rows, cols, 4))
    v[..., 0] = rng.integers(-1, 3, (rows, cols)).astype(float)
    v[..., 2] = rng.normal(0, 3, (rows, cols)) * 10.0 ** rng.integers(-6, 7, (rows, cols))
    v[..., 3] = rng.normal(0, 1, (rows, cols)).astype(np.float32)
    traj = rng.normal(200, 80, (6, 5, 2)).astype(np.float32)
    inp = f"{rows} {cols} {ps}\n" + " ".join(repr(float(x)) for x in v.ravel()) + "\n"
    inp += f"{traj.shape[0]} {traj.shape[1]}\n" + " ".join(repr(float(x)) for x in traj.ravel()) + "\n"
    cpp = str(tmp_path / "cpp")
    subprocess.run([str(exe), cpp], input=inp.encode(), check=True)
    py = str(tmp_path / "py")
    write_flow(v, py, ps)
    write_trajectories(list(traj), py + "_traj")
    lg = MotionLogger(py + "_log")
    lg.writeBoundingBox((10, 20, 30, 50), 12, 3)
    lg.writeContour([(1, 2), (3, 4), (-5, 6)], 13, 0)
    lg.close()
    for sfx in ("_h", "_f", "_traj", "_log"):
        assert open(cpp + sfx, "rb").read() == open(py + sfx, "rb").read(), sfx


@pytest.mark.gpu
@pytest.mark.parametrize("enc,skip", [("rgb8", 1), ("bgr8", 2), ("mono8", 1)])
def test_node_pair_path_matches_oracle(node_exe, tmp_path, mdx, oracle, enc, skip):
    """runOpticalFlow per processed frame, on the ring's last two rgb8 frames: the calculator's
    outputs (next_pts, status, mask, H, num_vectors), the node's Vec4d vector image as writeFlow
    writes it (optical_flow_calculator.cpp:509-541) and the comp mask on the build's own mask topic
    equal the oracle's.  Only reference-defined bytes are pinned: no topic under a reference name
    is published with content the reference does not define (~optical_flow_image's arrows are out
    of scope), and no motion.log is written (the reference logs cluster rectangles, node.cpp:431)."""
    from motion_detection_amd.formats import write_flow
    w, h, ps, mvs = 320, 240, 10, 1.0
    seq = []
    for s in range(3):
        a, b, _ = mdx.synth_pair(300 + s, w, h, 1 if enc == "mono8" else 3)
        seq += [a, b]
    if enc == "bgr8":
        seq = [x[:, :, ::-1].copy() for x in seq]
    frames = [(x, enc) for x in seq]
    p, out = run_node(node_exe, tmp_path, frames, live_path=False, egomotion=False, skip_frames=skip,
                      pixel_step=ps, min_vector_size=mvs)
    assert p.returncode == 0, p.stderr
    kept = kept_frames(len(frames), skip)
    ring_pairs = [(kept[i - 1], kept[i]) for i in range(1, len(kept))]   # trajectory_size 2
    assert f"processed {len(ring_pairs)} of {len(frames)}" in p.stdout, p.stdout
    for k, (i1, i2) in enumerate(ring_pairs):
        f1, f2 = to_rgb8(seq[i1], enc), to_rgb8(seq[i2], enc)
        ref = oracle.calculate_optical_flow(f1, f2, pixel_step=ps, min_vector_size=mvs)
        r = read_res(out / f"res_{k}.bin", live=False)
        assert r["num"] == ref["num_vectors"]
        assert np.array_equal(r["next_pts"].view(np.uint32), ref["next_pts"].view(np.uint32))
        assert np.array_equal(r["status"], ref["status"])
        assert np.array_equal(r["mask"], ref["mask"])
        assert np.array_equal(r["H"], ref["H"])
        mask_pub = np.fromfile(out / f"pub_{k}_motion_mask_image.rgb8", np.uint8).reshape(h, w, 3)
        assert np.array_equal(mask_pub, np.repeat(ref["mask"][:, :, None], 3, axis=2))
        assert not (out / f"pub_{k}_optical_flow_image.rgb8").exists()
        vi = vector_image(ref["vectors"], w, h, ps)
        pyf = str(tmp_path / f"py_flow_{k}")
        write_flow(vi, pyf, ps)
        for sfx in ("_h", "_f"):
            assert open(out / f"flow_{k}{sfx}", "rb").read() == open(pyf + sfx, "rb").read()
    assert not (out / "motion.log").exists()


@pytest.mark.gpu
@pytest.mark.parametrize("precision", [0, 1])
def test_node_live_path_matches_oracle(node_exe, tmp_path, mdx, oracle, precision):
    """The node's live branch: every ring frame through calculateOpticalFlowTrajectory, then
    fitSubspace on the complete trajectories with one rand() stream across frames (seeded), in
    double and in the reference's float arithmetic shape (subspace_precision=1)."""
    from motion_detection_amd.formats import write_trajectories
    w, h, ps, nm, sigma, seed = 320, 240, 10, 2, 0.5, 20141105
    a, b, _ = mdx.synth_pair(77, w, h, 3)
    c, d, _ = mdx.synth_pair(78, w, h, 3)
    seq = [a, b, a, b, a, c, d]
    frames = [(x, "rgb8") for x in seq]
    p, out = run_node(node_exe, tmp_path, frames, live_path=True, egomotion=True, num_motions=nm, sigma=sigma,
                      seed=seed, pixel_step=ps, subspace_precision=precision)
    assert p.returncode == 0, p.stderr
    ts = 2 * nm + 1
    st = oracle.rand_state(seed)
    k = 0
    for end in range(ts, len(seq) + 1):
        ring = seq[end - ts:end]
        ref = oracle.flow_trajectory(ring, pixel_step=ps)
        r = read_res(out / f"res_{k}.bin", live=True)
        assert r["num"] == ref["num_vectors"]
        full = np.array(ref["trajectories"], np.float32).reshape(-1, ts, 2)
        assert np.array_equal(r["traj"].view(np.uint32), full.view(np.uint32))
        if len(full):
            sub = oracle.fit_subspace(full, nm, sigma, st, precision)
            outl = full[sub["is_outlier"].astype(bool)][:, -2, :]
            assert np.array_equal(r["outliers"], outl.astype(np.float32))
            assert np.array_equal(r["columns"], sub["columns"][sub["columns"] >= 0])
        pyt = str(tmp_path / f"py_traj_{k}")
        write_trajectories(list(full), pyt)
        assert open(out / f"traj_{k}", "rb").read() == open(pyt, "rb").read()
        k += 1
    assert f"processed {k} of {len(seq)}" in p.stdout
