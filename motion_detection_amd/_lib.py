"""ctypes binding of libmdx.so (the C-ABI declared in include/mdx.h).

The library is built in-tree (motion_detection_amd/lib/libmdx.so) by
``motion_detection_amd.build()`` / ``__graft_entry__.build()``.  There is no CPU or
PyTorch fallback: if the library is missing, importing the compute API raises.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libmdx.so")
# developer hook: load an alternative build (e.g. scripts/lk_variants.sh timing-only variants)
if os.environ.get("MDX_LIB_PATH"):
    LIB_PATH = os.environ["MDX_LIB_PATH"]
CSRC = os.path.join(_HERE, "csrc")

MDX_OK = 0
MDX_EINVAL = -1
MDX_EHIP = -2
MDX_ENOMEM = -3
MDX_EDEGENERATE = 1

FMT_GRAY8, FMT_RGB8, FMT_BGR8 = 0, 1, 2
FIT_FIRST4, FIT_EXTERNAL, FIT_RANSAC = 0, 1, 2
SUBSPACE_F64, SUBSPACE_F32 = 0, 1

# every symbol include/mdx.h declares (checked by tests/test_abi.py)
EXPORTED = [
    "mdx_default_params", "mdx_grid_count", "mdx_create", "mdx_create_error", "mdx_destroy",
    "mdx_last_error", "mdx_set_params", "mdx_get_params", "mdx_stream", "mdx_device", "mdx_sync",
    "mdx_device_sync",
    "mdx_flow_warp_diff", "mdx_flow_warp_diff_batch_dev", "mdx_warp_diff_dev", "mdx_dev_alloc",
    "mdx_dev_free", "mdx_memcpy_h2d", "mdx_memcpy_d2h", "mdx_enable_timing", "mdx_timing_calls", "mdx_stage_ms",
    "mdx_synth_pair", "mdx_debug_copy", "mdx_band_flow_dev", "mdx_band_fit_warp_dev", "mdx_flow_trajectory",
    "mdx_srand", "mdx_rand", "mdx_fit_subspace", "mdx_device_pci", "mdx_build_info",
    "mdx_ring_push", "mdx_ring_trajectory", "mdx_ring_reset", "mdx_input_ready",
    "mdx_host_alloc", "mdx_host_free", "mdx_probe_stream3_dev", "mdx_lk_fallbacks",
    "mdx_debug_div32", "mdx_trajectory_layout", "mdx_abi_version", "mdx_params_size",
]
ABI_VERSION = 4   # include/mdx.h MDX_ABI_VERSION

# csrc/Makefile STAMPED: the files whose bytes the library's provenance stamp hashes, in order
STAMPED = ["Makefile", "mdx_internal.h", "mdx_api.cpp", "mdx_kernels.hip", "mdx_lk.hip", "mdx_warp.hip",
           "mdx_subspace.hip", "synth.cpp", os.path.join("..", "..", "include", "mdx.h")]


class MdxBandCand(C.Structure):
    """mdx_band_cand (include/mdx.h): one row band's accepted count and first four accepted points."""
    _fields_ = [("count", C.c_int32), ("n", C.c_int32), ("idx", C.c_int32 * 4), ("src", C.c_float * 8),
                ("dst", C.c_float * 8), ("pad_", C.c_int32 * 2)]


class MdxRandState(C.Structure):
    """mdx_rand_state (include/mdx.h): glibc rand() generator state."""
    _fields_ = [("x", C.c_uint32 * 34), ("pos", C.c_int32)]


BAND_CAND_BYTES = 96
assert C.sizeof(MdxBandCand) == BAND_CAND_BYTES


class MdxParams(C.Structure):
    _fields_ = [("win", C.c_int), ("max_level", C.c_int), ("max_iters", C.c_int), ("eps", C.c_double),
                ("min_eig", C.c_float), ("thresh", C.c_int), ("pixel_step", C.c_int),
                ("min_vector_size", C.c_double), ("fit_mode", C.c_int), ("subspace_precision", C.c_int),
                ("call_pipelining", C.c_int), ("ransac_iters", C.c_int), ("ransac_thresh", C.c_double),
                ("ransac_seed", C.c_uint32)]


class MdxError(RuntimeError):
    """Raised for every negative return code of the C-ABI."""


def build(force: bool = True) -> str:
    """Compile libmdx.so for gfx950 with hipcc (csrc/Makefile); force (default) rebuilds every
    object from the sources in the tree (make -B)."""
    cmd = ["make", "-s", "-C", CSRC] + (["-B"] if force else [])
    subprocess.run(cmd, check=True)
    return LIB_PATH


def source_sha256() -> str:
    """sha256 of the library's sources as csrc/Makefile stamps them into mdx_build_info()."""
    import hashlib
    h = hashlib.sha256()
    for f in STAMPED:
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def build_info() -> dict:
    """The loaded library's provenance stamp, and whether it matches the sources in this tree."""
    raw = lib().mdx_build_info().decode()
    kv = dict(part.split("=", 1) for part in raw.split())
    kv["matches_tree"] = kv.get("src_sha256") == source_sha256()
    return kv


_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MdxError(f"{LIB_PATH} is missing: build it with motion_detection_amd.build() "
                       "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    L = C.CDLL(LIB_PATH)
    vp, u8p, f32p, f64p, i32p = C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p
    if hasattr(L, "mdx_abi_version"):
        L.mdx_abi_version.argtypes = []
        L.mdx_abi_version.restype = C.c_int
        L.mdx_params_size.argtypes = []
        L.mdx_params_size.restype = C.c_size_t
        if L.mdx_abi_version() != ABI_VERSION or L.mdx_params_size() != C.sizeof(MdxParams):
            raise MdxError(f"{LIB_PATH}: ABI {L.mdx_abi_version()} / mdx_params {L.mdx_params_size()} B, this binding "
                           f"expects ABI {ABI_VERSION} / {C.sizeof(MdxParams)} B (rebuild the library)")
    elif not os.environ.get("MDX_LIB_PATH"):
        # only developer A/B builds of older revisions (MDX_LIB_PATH) may predate ABI 4
        raise MdxError(f"{LIB_PATH} predates ABI 4 (no mdx_abi_version): rebuild the library")
    L.mdx_default_params.argtypes = [C.POINTER(MdxParams)]
    L.mdx_default_params.restype = None
    L.mdx_grid_count.argtypes = [C.c_int, C.c_int, C.c_int]
    L.mdx_grid_count.restype = C.c_int
    L.mdx_create.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(MdxParams)]
    L.mdx_create.restype = vp
    L.mdx_create_error.argtypes = []
    L.mdx_create_error.restype = C.c_char_p
    L.mdx_destroy.argtypes = [vp]
    L.mdx_destroy.restype = C.c_int
    L.mdx_last_error.argtypes = [vp]
    L.mdx_last_error.restype = C.c_char_p
    L.mdx_set_params.argtypes = [vp, C.POINTER(MdxParams)]
    L.mdx_set_params.restype = C.c_int
    L.mdx_get_params.argtypes = [vp, C.POINTER(MdxParams)]
    L.mdx_get_params.restype = C.c_int
    L.mdx_stream.argtypes = [vp]
    L.mdx_stream.restype = vp
    L.mdx_device.argtypes = [vp]
    L.mdx_device.restype = C.c_int
    L.mdx_sync.argtypes = [vp]
    L.mdx_sync.restype = C.c_int
    L.mdx_device_pci.argtypes = [vp, C.c_char_p, C.c_int]
    L.mdx_device_pci.restype = C.c_int
    L.mdx_build_info.argtypes = []
    L.mdx_build_info.restype = C.c_char_p
    L.mdx_device_sync.argtypes = [vp]
    L.mdx_device_sync.restype = C.c_int
    if hasattr(L, "mdx_input_ready"):      # (absent from variant builds of older sources: A/B runs)
        L.mdx_input_ready.argtypes = [vp, vp]
        L.mdx_input_ready.restype = C.c_int
    L.mdx_flow_warp_diff.argtypes = [vp, u8p, u8p, C.c_int, C.c_int, C.c_int, C.c_int, f32p, u8p, f64p, u8p,
                                     f64p, f64p, C.POINTER(C.c_int)]
    L.mdx_flow_warp_diff.restype = C.c_int
    L.mdx_flow_warp_diff_batch_dev.argtypes = [vp, C.c_int, vp, vp, C.c_int, C.c_int, C.c_int, C.c_size_t, C.c_int,
                                               vp, vp, vp, vp, vp, vp, vp]
    L.mdx_flow_warp_diff_batch_dev.restype = C.c_int
    L.mdx_warp_diff_dev.argtypes = [vp, C.c_int, vp, vp, C.c_int, C.c_int, C.c_int, C.c_size_t, vp, vp]
    L.mdx_warp_diff_dev.restype = C.c_int
    if hasattr(L, "mdx_debug_div32"):
        L.mdx_debug_div32.argtypes = [vp, vp, vp, C.c_int]
        L.mdx_debug_div32.restype = C.c_int
    if hasattr(L, "mdx_lk_fallbacks"):
        L.mdx_lk_fallbacks.argtypes = [vp, C.POINTER(C.c_longlong)]
        L.mdx_lk_fallbacks.restype = C.c_int
    if hasattr(L, "mdx_trajectory_layout"):
        L.mdx_trajectory_layout.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_size_t)]
        L.mdx_trajectory_layout.restype = C.c_size_t
    if hasattr(L, "mdx_host_alloc"):
        L.mdx_host_alloc.argtypes = [C.c_size_t]
        L.mdx_host_alloc.restype = vp
        L.mdx_host_free.argtypes = [vp]
        L.mdx_host_free.restype = C.c_int
    if hasattr(L, "mdx_probe_stream3_dev"):
        L.mdx_probe_stream3_dev.argtypes = [vp, C.c_size_t, vp, vp, vp, C.c_int]
        L.mdx_probe_stream3_dev.restype = C.c_int
    L.mdx_dev_alloc.argtypes = [vp, C.c_size_t]
    L.mdx_dev_alloc.restype = vp
    L.mdx_dev_free.argtypes = [vp, vp]
    L.mdx_dev_free.restype = C.c_int
    L.mdx_memcpy_h2d.argtypes = [vp, vp, vp, C.c_size_t]
    L.mdx_memcpy_h2d.restype = C.c_int
    L.mdx_memcpy_d2h.argtypes = [vp, vp, vp, C.c_size_t]
    L.mdx_memcpy_d2h.restype = C.c_int
    L.mdx_enable_timing.argtypes = [vp, C.c_int]
    L.mdx_enable_timing.restype = C.c_int
    L.mdx_timing_calls.argtypes = [vp]
    L.mdx_timing_calls.restype = C.c_int
    L.mdx_stage_ms.argtypes = [vp, C.c_int, C.POINTER(C.c_float)]
    L.mdx_stage_ms.restype = C.c_int
    L.mdx_debug_copy.argtypes = [vp, C.c_int, vp, C.c_size_t]
    L.mdx_debug_copy.restype = C.c_int
    L.mdx_synth_pair.argtypes = [C.c_uint64, C.c_int, C.c_int, C.c_int, u8p, u8p, f64p, C.c_int]
    L.mdx_synth_pair.restype = C.c_int
    L.mdx_band_flow_dev.argtypes = [vp, vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp, vp, vp, vp]
    L.mdx_band_flow_dev.restype = C.c_int
    L.mdx_band_fit_warp_dev.argtypes = [vp, C.c_int, vp, C.c_int, C.c_int, vp, vp, vp]
    L.mdx_band_fit_warp_dev.restype = C.c_int
    L.mdx_flow_trajectory.argtypes = [vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, vp, vp, vp, vp,
                                      C.POINTER(C.c_int)]
    L.mdx_flow_trajectory.restype = C.c_int
    L.mdx_ring_push.argtypes = [vp, vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
    L.mdx_ring_push.restype = C.c_int
    L.mdx_ring_trajectory.argtypes = [vp, vp, vp, vp, vp, C.POINTER(C.c_int)]
    L.mdx_ring_trajectory.restype = C.c_int
    L.mdx_ring_reset.argtypes = [vp]
    L.mdx_ring_reset.restype = C.c_int
    L.mdx_srand.argtypes = [C.POINTER(MdxRandState), C.c_uint32]
    L.mdx_srand.restype = None
    L.mdx_rand.argtypes = [C.POINTER(MdxRandState)]
    L.mdx_rand.restype = C.c_int
    L.mdx_fit_subspace.argtypes = [vp, vp, C.c_int, C.c_int, C.c_int, C.c_double, C.POINTER(MdxRandState), vp, vp, vp,
                                   vp, C.POINTER(C.c_int)]
    L.mdx_fit_subspace.restype = C.c_int
    _lib = L
    return L


def default_params(**overrides) -> MdxParams:
    p = MdxParams()
    lib().mdx_default_params(C.byref(p))
    for k, v in overrides.items():
        if not hasattr(p, k):
            raise TypeError(f"unknown parameter {k!r}")
        setattr(p, k, v)
    return p
