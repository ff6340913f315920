"""CPU checks of the drop-in boundary: libmdx.so loads, exports every symbol include/mdx.h
declares, and its host-only entry points behave (no GPU needed; nothing here launches a kernel).

Boundary: the in-process seam OpticalFlowCalculator::calculateOpticalFlow
(reference common/include/motion_detection/optical_flow_calculator.h:19) -> mdx_flow_warp_diff.
"""
import ctypes as C
import json
import os
import re
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mdx.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)       # drop comments
    src = "\n".join(l for l in src.splitlines() if not l.lstrip().startswith("#"))
    return sorted(set(re.findall(r"\b(mdx_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    fns = header_functions()
    for f in ["mdx_create", "mdx_destroy", "mdx_last_error", "mdx_flow_warp_diff", "mdx_flow_warp_diff_batch_dev",
              "mdx_warp_diff_dev", "mdx_default_params", "mdx_grid_count"]:
        assert f in fns


def test_library_exports_every_header_symbol(mdx):
    L = mdx.lib()
    missing = [f for f in header_functions() if not hasattr(L, f)]
    assert not missing, missing


def test_binding_list_matches_header(mdx):
    from motion_detection_amd import _lib
    assert sorted(_lib.EXPORTED) == header_functions()


def test_exports_are_plain_c(mdx):
    # extern "C": no mangled mdx symbols in the dynamic table
    out = subprocess.run(["nm", "-D", "--defined-only", mdx.LIB_PATH], capture_output=True, text=True, check=True).stdout
    syms = {l.split()[-1] for l in out.splitlines() if l.strip()}
    for f in header_functions():
        assert f in syms, f


def test_abi_version_and_params_size(mdx):
    """mdx_abi_version / mdx_params_size (ABI 4) equal the header's MDX_ABI_VERSION and the
    binding's mdx_params layout; the binding refuses a library that disagrees."""
    hdr = open(os.path.join(ROOT, "include", "mdx.h")).read()
    ver = int(re.search(r"#define MDX_ABI_VERSION (\d+)", hdr).group(1))
    from motion_detection_amd import _lib
    L = _lib.lib()
    assert L.mdx_abi_version() == ver == _lib.ABI_VERSION
    assert L.mdx_params_size() == C.sizeof(_lib.MdxParams) == 80


def test_default_params_are_reference_constants(mdx):
    from motion_detection_amd import _lib
    p = _lib.MdxParams()
    mdx.lib().mdx_default_params(C.byref(p))
    # optical_flow_calculator.cpp:40-44,71,127; node.cpp:29,44
    assert (p.win, p.max_level, p.max_iters) == (40, 5, 10)
    assert p.eps == pytest.approx(0.03) and p.min_eig == pytest.approx(1e-3)
    assert (p.thresh, p.pixel_step, p.fit_mode) == (190, 10, _lib.FIT_FIRST4)
    assert p.min_vector_size == 1.0


@pytest.mark.parametrize("w,h,ps", [(640, 480, 10), (1920, 1080, 10), (3840, 2160, 10), (1920, 1080, 3), (25, 17, 10),
                                    (1, 1, 1), (0, 10, 10), (10, 10, 0)])
def test_grid_count(mdx, w, h, ps):
    exp = 0 if min(w, h, ps) <= 0 else -(-w // ps) * -(-h // ps)
    assert mdx.lib().mdx_grid_count(w, h, ps) == exp


def test_null_context_is_einval(mdx):
    from motion_detection_amd import _lib
    L = mdx.lib()
    assert L.mdx_destroy(None) == _lib.MDX_EINVAL
    assert L.mdx_sync(None) == _lib.MDX_EINVAL
    assert L.mdx_last_error(None) == b"null context"
    buf = np.zeros(16, np.uint8)
    p = buf.ctypes.data_as(C.c_void_p)
    assert L.mdx_flow_warp_diff(None, p, p, 4, 4, 4, 0, None, None, None, None, None, None, None) == _lib.MDX_EINVAL
    assert L.mdx_warp_diff_dev(None, 1, p, p, 4, 4, 4, 16, p, p) == _lib.MDX_EINVAL


def test_create_rejects_bad_params(mdx):
    from motion_detection_amd import _lib
    L = mdx.lib()
    p = _lib.default_params(win=21)
    assert not L.mdx_create(0, 64, 64, 1, C.byref(p))
    assert b"win" in L.mdx_create_error()
    p = _lib.default_params(pixel_step=0)
    assert not L.mdx_create(0, 64, 64, 1, C.byref(p))
    assert b"pixel_step" in L.mdx_create_error()


def test_create_without_gpu_fails_cleanly(mdx):
    L = mdx.lib()
    h = L.mdx_create(0, 64, 64, 1, None)
    if h:   # a GPU box running the CPU suite
        L.mdx_destroy(h)
        pytest.skip("a HIP device is visible")
    assert b"device" in L.mdx_create_error()


def test_synth_generator_is_deterministic(mdx):
    """mdx_synth_pair must reproduce the committed golden inputs byte for byte."""
    g = np.load(os.path.join(ROOT, "tests", "golden", "synth_160x120_gray.npz"))
    a, b, H = mdx.synth_pair(20141105, 160, 120, 1)
    assert np.array_equal(a, g["img1"]) and np.array_equal(b, g["img2"])
    a4, b4, _ = mdx.synth_pair(20141105, 160, 120, 1, nthreads=4)
    assert np.array_equal(a, a4) and np.array_equal(b, b4)
    g = np.load(os.path.join(ROOT, "tests", "golden", "synth_160x120_rgb.npz"))
    a, b, _ = mdx.synth_pair(20141107, 160, 120, 3)
    assert np.array_equal(a, g["img1"]) and np.array_equal(b, g["img2"])


def test_synth_true_homography(mdx):
    # rotation 0.5 deg about the centre, scale 1.01, translation (3.2, -1.7)  
    _, _, H = mdx.synth_pair(1, 200, 100, 1)
    th = np.deg2rad(0.5)
    R = 1.01 * np.array([[np.cos(th), -np.sin(th)], [np.sin(th), np.cos(th)]])
    c = np.array([100.0, 50.0])
    assert np.allclose(H[:2, :2], R, atol=1e-12)
    assert np.allclose(H[:2, 2], c - R @ c + [3.2, -1.7], atol=1e-9)
    assert np.array_equal(H[2], [0, 0, 1])


def test_missing_library_fails_loudly():
    """No CPU fallback: a missing libmdx.so raises instead of silently computing on the host."""
    code = ("import motion_detection_amd as m\n"
            "try:\n    m.lib()\nexcept m.MdxError as e:\n    print('RAISED', 'no CPU fallback' in str(e))\n")
    env = dict(os.environ, MDX_LIB_PATH=os.path.join(ROOT, "does_not_exist", "libmdx.so"))
    out = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert "RAISED True" in out.stdout, out.stdout + out.stderr


def test_golden_manifest_covers_fixtures():
    man = json.load(open(os.path.join(ROOT, "tests", "golden", "manifest.json")))
    for name in man:
        assert os.path.exists(os.path.join(ROOT, "tests", "golden", name + ".npz"))


def test_library_built_from_the_tree_sources(mdx):
    """Provenance: the loaded libmdx.so carries the sha256 of the sources it was compiled from
    (csrc/Makefile stamps it); it must equal the hash of the sources in this tree, so a stale or
    foreign library cannot pass the GPU tests."""
    from motion_detection_amd import _lib
    if os.environ.get("MDX_LIB_PATH"):
        pytest.skip("variant library selected by MDX_LIB_PATH")
    info = _lib.build_info()
    assert info["arch"] == "gfx950"
    assert info["matches_tree"], (info, _lib.source_sha256())
