"""Python host over the C-ABI: a device context per camera stream / GPU.

Thin ownership wrapper around ``mdx_ctx`` (include/mdx.h).  Numpy arrays on the host
side, raw device pointers (ints) for the zero-copy batched entry; no torch types.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import MdxError, lib


def _ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def grid_count(w: int, h: int, pixel_step: int) -> int:
    return lib().mdx_grid_count(w, h, pixel_step)


def grid_points(w: int, h: int, pixel_step: int) -> np.ndarray:
    """Grid of the reference (optical_flow_calculator.cpp:56-64): x-major, float32 (n, 2)."""
    xs = np.arange(0, w, pixel_step, dtype=np.float32)
    ys = np.arange(0, h, pixel_step, dtype=np.float32)
    gx, gy = np.meshgrid(xs, ys, indexing="ij")
    return np.stack([gx.ravel(), gy.ravel()], 1)


@dataclass
class FlowResult:
    num_vectors: int        # reference return value
    next_pts: np.ndarray    # (npts, 2) float32, LK output positions, x-major grid order
    status: np.ndarray      # (npts,) uint8
    vectors: np.ndarray     # (npts, 4) float64: (x, y, dx, dy) / (x, y, 0, 0) / (-1, -1, 0, 0)
    mask: np.ndarray | None  # (h, w) uint8 or None
    H: np.ndarray           # (3, 3) float64 (zeros when no fit)
    code: int               # MDX_OK or MDX_EDEGENERATE


@dataclass
class TrajectoryResult:
    num_vectors: int        # reference return value (last pass)
    traj: np.ndarray        # (npts, nimg, 2) float32: grid point, then each accepted move
    traj_len: np.ndarray    # (npts,) int32: entries of traj in use (complete iff == nimg)
    start_pts: np.ndarray   # (npts, 2) float32: points entering the last pass
    vectors: np.ndarray     # (npts, 4) float64: the last pass's Vec4d per point

    @property
    def trajectories(self) -> list:
        """The reference's output list (optical_flow_calculator.cpp:244-249): the complete ones,
        in grid order, each (nimg, 2)."""
        nimg = self.traj.shape[1]
        return [self.traj[i] for i in np.nonzero(self.traj_len == nimg)[0]]


@dataclass
class SubspaceResult:
    columns: np.ndarray         # (4*num_motions,) int32: the winning sample (-1: no hypothesis had an inlier)
    is_outlier: np.ndarray      # (ntraj,) uint8
    residuals: np.ndarray       # (ntraj,) float64, the winner's
    outlier_points: np.ndarray  # (n_outliers, 2) float32: each outlier's second-to-last point


class Context:
    """One device context (mdx_ctx): workspace sized at creation, one HIP stream."""

    def __init__(self, device: int = 0, max_w: int = 1920, max_h: int = 1080, max_batch: int = 1, **params):
        self._p = _lib.default_params(**params)
        h = lib().mdx_create(device, max_w, max_h, max_batch, C.byref(self._p))
        if not h:
            raise MdxError("mdx_create failed: " + lib().mdx_create_error().decode())
        self._h = C.c_void_p(h)
        self._ring_hold = []    # frames whose asynchronous ring push may still be reading them

    # -- lifetime
    def close(self):
        if getattr(self, "_h", None):
            lib().mdx_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def device(self) -> int:
        return lib().mdx_device(self._h)

    def device_pci(self) -> str:
        """PCI bus id of the context's device (distinct per physical GPU)."""
        buf = C.create_string_buffer(64)
        self._check(lib().mdx_device_pci(self._h, buf, 64))
        return buf.value.decode()

    def _check(self, rc: int) -> int:
        if rc < 0:
            raise MdxError(f"mdx error {rc}: {lib().mdx_last_error(self._h).decode()}")
        return rc

    # -- params
    @property
    def params(self) -> _lib.MdxParams:
        p = _lib.MdxParams()
        self._check(lib().mdx_get_params(self._h, C.byref(p)))
        return p

    def set_params(self, **kw):
        p = self.params
        for k, v in kw.items():
            setattr(p, k, v)
        self._check(lib().mdx_set_params(self._h, C.byref(p)))

    # -- host entry (drop-in for calculateOpticalFlow)
    def flow_warp_diff(self, img1: np.ndarray, img2: np.ndarray, fmt: int | None = None, want_mask: bool = True,
                       H_external: np.ndarray | None = None) -> FlowResult:
        img1 = np.ascontiguousarray(img1, dtype=np.uint8)
        img2 = np.ascontiguousarray(img2, dtype=np.uint8)
        if img1.shape != img2.shape:
            raise ValueError("frames must have the same shape")
        h, w = img1.shape[:2]
        if fmt is None:
            fmt = _lib.FMT_GRAY8 if img1.ndim == 2 else _lib.FMT_RGB8
        p = self.params
        n = grid_count(w, h, p.pixel_step)
        nextp = np.zeros((n, 2), np.float32)
        status = np.zeros(n, np.uint8)
        vec = np.zeros((n, 4), np.float64)
        mask = np.zeros((h, w), np.uint8) if want_mask else None
        H = np.zeros(9, np.float64)
        Hx = None if H_external is None else np.ascontiguousarray(H_external, dtype=np.float64).ravel()
        num = C.c_int(0)
        rc = self._check(lib().mdx_flow_warp_diff(self._h, _ptr(img1), _ptr(img2), w, h, img1.strides[0], fmt,
                                                  _ptr(nextp), _ptr(status), _ptr(vec), _ptr(mask), _ptr(H), _ptr(Hx),
                                                  C.byref(num)))
        return FlowResult(num.value, nextp, status, vec, mask, H.reshape(3, 3), rc)

    # -- trajectory tracking (drop-in for calculateOpticalFlowTrajectory)
    def flow_trajectory(self, images, fmt: int | None = None) -> "TrajectoryResult":
        imgs = [np.ascontiguousarray(im, dtype=np.uint8) for im in images]
        if len(imgs) < 2 or any(im.shape != imgs[0].shape for im in imgs):
            raise ValueError("need >= 2 frames of one shape")
        h, w = imgs[0].shape[:2]
        if fmt is None:
            fmt = _lib.FMT_GRAY8 if imgs[0].ndim == 2 else _lib.FMT_RGB8
        nimg = len(imgs)
        n = grid_count(w, h, self.params.pixel_step)
        traj = np.zeros((n, nimg, 2), np.float32)
        tlen = np.zeros(n, np.int32)
        start = np.zeros((n, 2), np.float32)
        vec = np.zeros((n, 4), np.float64)
        arr = (C.c_void_p * nimg)(*[im.ctypes.data for im in imgs])
        num = C.c_int(0)
        self._check(lib().mdx_flow_trajectory(self._h, arr, nimg, w, h, imgs[0].strides[0], fmt, _ptr(traj),
                                              _ptr(tlen), _ptr(start), _ptr(vec), C.byref(num)))
        return TrajectoryResult(num.value, traj, tlen, start, vec)

    # -- resident frame ring (the node's raw_images_ deque kept in HBM: mdx_ring_*)
    def ring_push(self, image: np.ndarray, keep: int, fmt: int | None = None) -> int:
        """Append one frame (pyramided once, on the device) and keep at most `keep` frames.
        Returns the number of frames held."""
        im = np.ascontiguousarray(image, dtype=np.uint8)
        h, w = im.shape[:2]
        if fmt is None:
            fmt = _lib.FMT_GRAY8 if im.ndim == 2 else _lib.FMT_RGB8
        n = self._check(lib().mdx_ring_push(self._h, _ptr(im), w, h, im.strides[0], fmt, int(keep)))
        # the upload is queued, not done (include/mdx.h): hold the frame until the next
        # ring_trajectory / sync returns
        self._ring_hold.append(im)
        return n

    def ring_trajectory(self, w: int, h: int, nimg: int, out: "TrajectoryResult | None" = None) -> "TrajectoryResult":
        """calculateOpticalFlowTrajectory over the ring's `nimg` frames (w x h).  `out`: arrays to
        fill (e.g. from trajectory_buffers(pinned=True)), reused across callbacks."""
        n = grid_count(w, h, self.params.pixel_step)
        if out is None:
            out = self.trajectory_buffers(w, h, nimg)
        traj, tlen, start, vec = out.traj, out.traj_len, out.start_pts, out.vectors
        num = C.c_int(0)
        assert traj.shape == (n, nimg, 2) and tlen.shape == (n,) and start.shape == (n, 2) and vec.shape == (n, 4)
        rc = lib().mdx_ring_trajectory(self._h, _ptr(traj), _ptr(tlen), _ptr(start), _ptr(vec), C.byref(num))
        if rc < 0:
            # the uploads queued by earlier ring_push calls may still read the held frames: release
            # them only once the stream has drained
            lib().mdx_sync(self._h)
        self._ring_hold.clear()
        self._check(rc)
        out.num_vectors = num.value
        return out

    def trajectory_buffers(self, w: int, h: int, nimg: int, pinned: bool = False) -> "TrajectoryResult":
        """Output arrays of a trajectory call; pinned=True puts them in one page-locked block laid
        out as mdx_trajectory_layout says, so the call reads them back with one copy."""
        n = grid_count(w, h, self.params.pixel_step)
        if not pinned:
            return TrajectoryResult(0, np.zeros((n, nimg, 2), np.float32), np.zeros((n,), np.int32),
                                    np.zeros((n, 2), np.float32), np.zeros((n, 4), np.float64))
        if not hasattr(lib(), "mdx_trajectory_layout"):
            return TrajectoryResult(0, host_empty((n, nimg, 2), np.float32), host_empty((n,), np.int32),
                                    host_empty((n, 2), np.float32), host_empty((n, 4), np.float64))
        off = (C.c_size_t * 4)()
        total = int(lib().mdx_trajectory_layout(n, nimg, off))
        blk = host_empty((total,), np.uint8)

        def part(o, shape, dt):
            cnt = int(np.prod(shape))
            return blk[o:o + cnt * np.dtype(dt).itemsize].view(dt).reshape(shape)
        return TrajectoryResult(0, part(off[0], (n, nimg, 2), np.float32), part(off[3], (n,), np.int32),
                                part(off[1], (n, 2), np.float32), part(off[2], (n, 4), np.float64))

    def ring_reset(self) -> None:
        self._check(lib().mdx_ring_reset(self._h))

    # -- trajectory subspace RANSAC (drop-in for OutlierDetector::fitSubspace)
    def fit_subspace(self, traj: np.ndarray, num_motions: int, sigma: float, rng: "_lib.MdxRandState") -> "SubspaceResult":
        traj = np.ascontiguousarray(traj, dtype=np.float32)
        if traj.ndim != 3 or traj.shape[2] != 2:
            raise ValueError("traj must be (ntraj, traj_len, 2)")
        N, T = traj.shape[:2]
        d = 4 * num_motions
        cols = np.full(d, -1, np.int32)
        out = np.zeros(N, np.uint8)
        res = np.zeros(N, np.float64)
        pts = np.zeros((N, 2), np.float32)
        nout = C.c_int(0)
        self._check(lib().mdx_fit_subspace(self._h, _ptr(traj), N, T, int(num_motions), float(sigma), C.byref(rng),
                                           _ptr(cols), _ptr(out), _ptr(res), _ptr(pts), C.byref(nout)))
        return SubspaceResult(cols, out, res, pts[:nout.value].copy())

    # -- device entries (pointers are ints, e.g. torch.Tensor.data_ptr())
    def flow_warp_diff_batch_dev(self, batch: int, d_img1: int, d_img2: int, w: int, h: int, stride: int,
                                 frame_stride: int, fmt: int = _lib.FMT_GRAY8, d_next_pts: int = 0, d_status: int = 0,
                                 d_vectors: int = 0, d_mask: int = 0, d_H: int = 0, d_H_external: int = 0,
                                 d_num_vectors: int = 0) -> int:
        v = lambda x: C.c_void_p(x) if x else None  # noqa: E731
        return self._check(lib().mdx_flow_warp_diff_batch_dev(
            self._h, batch, v(d_img1), v(d_img2), w, h, stride, frame_stride, fmt, v(d_next_pts), v(d_status),
            v(d_vectors), v(d_mask), v(d_H), v(d_H_external), v(d_num_vectors)))

    def warp_diff_dev(self, batch: int, d_gray1: int, d_gray2: int, w: int, h: int, stride: int, frame_stride: int,
                      d_H: int, d_mask: int) -> int:
        return self._check(lib().mdx_warp_diff_dev(self._h, batch, C.c_void_p(d_gray1), C.c_void_p(d_gray2), w, h,
                                                   stride, frame_stride, C.c_void_p(d_H), C.c_void_p(d_mask)))

    def probe_stream3_dev(self, n: int, d_a: int, d_b: int, d_mask: int, thresh: int = 190) -> int:
        """Memory-ceiling probe of k_warp_diff's 3 B/px access mix (include/mdx.h)."""
        return self._check(lib().mdx_probe_stream3_dev(self._h, n, C.c_void_p(d_a), C.c_void_p(d_b),
                                                       C.c_void_p(d_mask), thresh))

    # -- row-tiled path (one pair split by rows over ranks; include/mdx.h mdx_band_*)
    def band_flow_dev(self, d_img1: int, d_img2: int, w: int, h: int, stride: int, fmt: int, y0: int, y1: int,
                      d_next_pts: int, d_status: int, d_cand: int, d_vectors: int = 0) -> int:
        v = lambda x: C.c_void_p(x) if x else None  # noqa: E731
        return self._check(lib().mdx_band_flow_dev(self._h, v(d_img1), v(d_img2), w, h, stride, fmt, y0, y1,
                                                   v(d_next_pts), v(d_status), v(d_vectors), v(d_cand)))

    def band_fit_warp_dev(self, nrec: int, d_cands: int, y0: int, y1: int, d_mask_band: int, d_H: int = 0,
                          d_num_vectors: int = 0) -> int:
        v = lambda x: C.c_void_p(x) if x else None  # noqa: E731
        return self._check(lib().mdx_band_fit_warp_dev(self._h, nrec, v(d_cands), y0, y1, v(d_mask_band), v(d_H),
                                                       v(d_num_vectors)))

    def input_ready(self, hip_event: int):
        """The next device-entry call waits for this hipEvent_t (an int handle) before reading its
        input frames (include/mdx.h mdx_input_ready; one-shot)."""
        self._check(lib().mdx_input_ready(self._h, C.c_void_p(hip_event) if hip_event else None))

    def sync(self):
        self._check(lib().mdx_sync(self._h))
        self._ring_hold.clear()

    def device_sync(self):
        self._check(lib().mdx_device_sync(self._h))

    def lk_fallbacks(self) -> dict:
        """LK level-dataflow fallbacks since creation, as of the last sync (include/mdx.h
        mdx_lk_fallbacks): waits that gave up and levels recomputed -- statistics, not errors."""
        if not hasattr(lib(), "mdx_lk_fallbacks"):     # (variant builds of older sources: A/B runs)
            return None
        v = (C.c_longlong * 3)()
        self._check(lib().mdx_lk_fallbacks(self._h, v))
        return {"group_giveups": v[0], "gate_giveups": v[1], "levels_recomputed": v[2]}

    @property
    def stream(self) -> int:
        return lib().mdx_stream(self._h) or 0

    def enable_timing(self, on: bool = True):
        self._check(lib().mdx_enable_timing(self._h, int(on)))

    def stage_ms(self) -> dict:
        """Per-stage device ms summed over the calls since enable_timing(); 'calls' = count."""
        names = ["gray_pad", "pyrdown", "scharr", "lk", "classify_fit", "warp_diff", "total"]
        out = {"calls": lib().mdx_timing_calls(self._h)}
        for i, nm in enumerate(names):
            ms = C.c_float(0)
            self._check(lib().mdx_stage_ms(self._h, i, C.byref(ms)))
            out[nm] = ms.value
        return out

    # -- device memory helpers (no torch needed)
    def dev_alloc(self, nbytes: int) -> int:
        p = lib().mdx_dev_alloc(self._h, nbytes)
        if not p:
            raise MdxError(lib().mdx_last_error(self._h).decode())
        return p

    def dev_free(self, ptr: int):
        self._check(lib().mdx_dev_free(self._h, C.c_void_p(ptr)))

    def h2d(self, dst: int, src: np.ndarray):
        src = np.ascontiguousarray(src)
        self._check(lib().mdx_memcpy_h2d(self._h, C.c_void_p(dst), _ptr(src), src.nbytes))

    def d2h(self, dst: np.ndarray, src: int):
        self._check(lib().mdx_memcpy_d2h(self._h, _ptr(dst), C.c_void_p(src), dst.nbytes))


class _HostBlock:
    """Owner of one mdx_host_alloc block; freed when the last array viewing it goes away."""

    def __init__(self, nbytes: int):
        self.nbytes = max(1, nbytes)
        self.ptr = lib().mdx_host_alloc(self.nbytes)
        if not self.ptr:
            raise MdxError(f"mdx_host_alloc({nbytes}) failed")

    def __del__(self):
        try:
            lib().mdx_host_free(C.c_void_p(self.ptr))
        except Exception:
            pass


class PinnedArray(np.ndarray):
    """numpy array over page-locked host memory; views keep the block alive through their base."""
    _blk = None


def host_empty(shape, dtype=np.uint8) -> np.ndarray:
    """A numpy array in page-locked host memory (include/mdx.h mdx_host_alloc): frames and outputs
    in it cross PCIe by DMA at full rate.  The block is freed with the array."""
    dtype = np.dtype(dtype)
    n = int(np.prod(shape)) * dtype.itemsize
    blk = _HostBlock(n)
    raw = (C.c_uint8 * blk.nbytes).from_address(blk.ptr)
    # the block hangs off the lowest buffer object: numpy collapses a view's base chain down to
    # `raw` (np.asarray, .view(np.ndarray) and ascontiguousarray skip the PinnedArray), so every
    # view of the memory keeps it alive
    raw._blk = blk
    arr = np.frombuffer(raw, dtype=np.uint8, count=n).view(dtype).reshape(shape).view(PinnedArray)
    arr._blk = blk
    return arr


def synth_pair(seed: int, w: int, h: int, channels: int = 1, nthreads: int = 0):
    """Deterministic synthetic frame pair.  Returns (img1, img2, H_true)."""
    shape = (h, w) if channels == 1 else (h, w, channels)
    a = np.empty(shape, np.uint8)
    b = np.empty(shape, np.uint8)
    H = np.zeros(9, np.float64)
    rc = lib().mdx_synth_pair(seed, w, h, channels, _ptr(a), _ptr(b), _ptr(H), nthreads)
    if rc != 0:
        raise MdxError(f"mdx_synth_pair failed ({rc})")
    return a, b, H.reshape(3, 3)
