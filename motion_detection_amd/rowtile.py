"""Row-tiled path: one frame pair split by rows over several GPUs.

The reference runs the whole frame in one ``calculateOpticalFlow`` call
(common/src/optical_flow_calculator.cpp:30-130).  Its only frame-global step is the
getPerspectiveTransform input, the first four accepted vectors in x-major grid order
(:118-120); everything else is per grid point (LK, :71-117) or per pixel (warp + diff, :124-127).
So a frame splits by rows with one small exchange:

1. each rank runs ``mdx_band_flow_dev`` for its band of rows -> its points' flow and one
   96-byte ``mdx_band_cand`` record (the band's accepted count and first four accepted points);
2. the ranks all-gather the records (RCCL over xGMI in ``bench.py``; any transport works);
3. each rank runs ``mdx_band_fit_warp_dev`` -> the identical FP64 fit on every rank (the four
   smallest indices over all records) and the mask rows of its band.

``merge_records`` is the host statement of step 3's merge; the CPU tests check it against the
oracle's full-frame first four, and the GPU tests check the device path against the full path.
"""
from __future__ import annotations

import ctypes as C
from typing import Callable, Sequence

import numpy as np

from ._lib import BAND_CAND_BYTES, MdxBandCand

# numpy view of mdx_band_cand (include/mdx.h)
BAND_CAND_DTYPE = np.dtype([("count", "<i4"), ("n", "<i4"), ("idx", "<i4", 4), ("src", "<f4", 8),
                            ("dst", "<f4", 8), ("pad_", "<i4", 2)])
assert BAND_CAND_DTYPE.itemsize == BAND_CAND_BYTES == C.sizeof(MdxBandCand)


def band_rows(h: int, nbands: int, b: int) -> tuple[int, int]:
    """Rows [y0, y1) of band b when h rows are split into nbands contiguous, balanced bands."""
    if not 0 <= b < nbands or nbands > h:
        raise ValueError(f"band {b} of {nbands} over {h} rows")
    return (h * b) // nbands, (h * (b + 1)) // nbands


def band_grid_rows(y0: int, y1: int, pixel_step: int) -> tuple[int, int]:
    """Grid rows gy with gy * pixel_step in [y0, y1) (the band's points)."""
    return -(-y0 // pixel_step), -(-y1 // pixel_step)


def band_record(next_pts: np.ndarray, status: np.ndarray, w: int, h: int, pixel_step: int,
                min_vector_size: float, y0: int, y1: int) -> np.ndarray:
    """Host statement of the band record (k_band_record) from full-frame LK outputs.

    Accepted = status and (|dx| > mvs or |dy| > mvs) with float differences, as the
    classification at optical_flow_calculator.cpp:78-117.
    """
    ny = -(-h // pixel_step)
    n = next_pts.shape[0]
    idx = np.arange(n)
    gx, gy = idx // ny, idx % ny
    sx = (gx * pixel_step).astype(np.float32)
    sy = (gy * pixel_step).astype(np.float32)
    dx = next_pts[:, 0].astype(np.float32) - sx
    dy = next_pts[:, 1].astype(np.float32) - sy
    gy0, gy1 = band_grid_rows(y0, y1, pixel_step)
    acc = (status != 0) & ((np.abs(dx).astype(np.float64) > min_vector_size) |
                           (np.abs(dy).astype(np.float64) > min_vector_size)) & (gy >= gy0) & (gy < gy1)
    sel = np.nonzero(acc)[0]
    rec = np.zeros(1, BAND_CAND_DTYPE)
    rec["count"] = sel.size
    k = min(sel.size, 4)
    rec["n"] = k
    rec["idx"][0] = -1
    for r in range(k):
        i = sel[r]
        rec["idx"][0, r] = i
        rec["src"][0, 2 * r:2 * r + 2] = (sx[i], sy[i])
        rec["dst"][0, 2 * r:2 * r + 2] = next_pts[i]
    return rec


def merge_records(records: np.ndarray) -> tuple[int, np.ndarray, np.ndarray, np.ndarray]:
    """Host statement of k_band_fit's merge: (num_vectors, first-4 idx, src (4,2), dst (4,2)).

    Bands partition the points and each record lists its band's first accepted points in
    x-major order, so the four smallest indices over all records are the frame's first four.
    """
    records = np.asarray(records, BAND_CAND_DTYPE).ravel()
    total = int(records["count"].sum())
    cand = []
    for rec in records:
        for r in range(int(rec["n"])):
            cand.append((int(rec["idx"][r]), rec["src"][2 * r:2 * r + 2], rec["dst"][2 * r:2 * r + 2]))
    cand.sort(key=lambda t: t[0])
    cand = cand[:4]
    idx = np.array([c[0] for c in cand], np.int64)
    src = np.array([c[1] for c in cand], np.float32).reshape(-1, 2)
    dst = np.array([c[2] for c in cand], np.float32).reshape(-1, 2)
    return total, idx, src, dst


class RowTiledPair:
    """Drive the three steps for one rank on its context (device pointers are ints).

    ``allgather(local: bytes) -> Sequence[bytes]`` returns every rank's record (any order) and is
    the only communication.  Buffers: d_next_pts [npts][2] f32, d_status [npts] u8 (full-frame;
    this rank writes its band's entries), d_cand (96 B), d_cands (nranks * 96 B), d_mask_band
    ((y1 - y0) * w u8), d_H (9 f64), d_num (i32).
    """

    def __init__(self, ctx, w: int, h: int, fmt: int, rank: int, nranks: int):
        self.ctx, self.w, self.h, self.fmt = ctx, w, h, fmt
        self.rank, self.nranks = rank, nranks
        self.y0, self.y1 = band_rows(h, nranks, rank)

    def flow(self, d_img1: int, d_img2: int, stride: int, d_next_pts: int, d_status: int, d_cand: int,
             d_vectors: int = 0) -> int:
        return self.ctx.band_flow_dev(d_img1, d_img2, self.w, self.h, stride, self.fmt, self.y0, self.y1, d_next_pts,
                                      d_status, d_cand, d_vectors)

    def fit_warp(self, d_cands: int, d_mask_band: int, d_H: int = 0, d_num: int = 0) -> int:
        return self.ctx.band_fit_warp_dev(self.nranks, d_cands, self.y0, self.y1, d_mask_band, d_H, d_num)


def gather_records_host(local: bytes, allgather: Callable[[bytes], Sequence[bytes]]) -> bytes:
    """All-gather one 96-byte record per rank through a host callable; returns the concatenation."""
    if len(local) != BAND_CAND_BYTES:
        raise ValueError("a band record is 96 bytes")
    parts = list(allgather(local))
    if any(len(p) != BAND_CAND_BYTES for p in parts):
        raise ValueError("bad record size from a peer")
    return b"".join(parts)
