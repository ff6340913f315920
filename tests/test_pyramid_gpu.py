"""GPU parity of the front end alone: every padded pyramid level the HIP path leaves in HBM
(k_front = gray + pad + level-1 pyrDown, then k_front's level mode for the coarser levels) equals
the oracle's buildOpticalFlowPyramid images byte for byte, borders included (lkpyramid.cpp:
buildOpticalFlowPyramid with BORDER_REFLECT_101, withDerivatives; reference call at
optical_flow_calculator.cpp:71).  Both the split-frame launch of the pair path (first frames,
then second frames) and the both-frames launch of the trajectory path are covered; the band
heights 4 (1080p), 2 (4K level 0) and 1 (a 12K-wide row, > 64 KB of LDS) all run.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

KPAD, KXOFF, KWIN = 40, 64, 40


def geometry(w, h, max_level):
    levels, off = [], 0
    sw, sh = w, h
    for _ in range(max_level + 1):
        pitch = (KXOFF + sw + KPAD + 16 + 63) // 64 * 64
        rows = KPAD + sh + KPAD
        levels.append((sw, sh, pitch, off))
        off += pitch * rows
        sw, sh = (sw + 1) // 2, (sh + 1) // 2
        if sw <= KWIN or sh <= KWIN:
            break
    return levels, (off + 255) // 256 * 256


def padded_levels(slab, levels, pair, img_bytes):
    out = []
    for sw, sh, pitch, off in levels:
        base = pair * img_bytes + off
        a = slab[base:base + pitch * (sh + 2 * KPAD)].reshape(sh + 2 * KPAD, pitch)
        out.append(a[:, KXOFF - KPAD:KXOFF + sw + KPAD])
    return out


def frames(w, h, ch, seed):
    rng = np.random.default_rng(seed)
    shape = (h, w) if ch == 1 else (h, w, 3)
    a = rng.integers(0, 256, shape, dtype=np.uint8)
    b = np.roll(a, (3, -2), (0, 1))
    return a, b


def check(mdx, c, oracle, gray_frames, which_slabs, npairs):
    levels, img_bytes = geometry(gray_frames[0].shape[1], gray_frames[0].shape[0], c.params.max_level)
    for slab_id, frames_of_slab in which_slabs:
        slab = np.empty(img_bytes * npairs, np.uint8)
        mdx.lib().mdx_debug_copy(c._h, slab_id, slab.ctypes.data, slab.nbytes)
        for pair in range(npairs):
            got = padded_levels(slab, levels, pair, img_bytes)
            ml, ref, _ = oracle.build_pyramid(frames_of_slab[pair], KWIN, c.params.max_level, with_deriv=False)
            assert len(ref) == len(got), (len(ref), len(got))
            for lv, (g, r) in enumerate(zip(got, ref)):
                bad = np.argwhere(g != r)
                assert bad.size == 0, f"slab {slab_id} pair {pair} level {lv}: {len(bad)} bytes differ, first {bad[:4]}"


CASES = [
    (160, 120, 1, 1),
    (333, 241, 1, 2),
    (81, 83, 1, 3),
    (320, 240, 3, 4),
    (641, 483, 3, 5),
    (1920, 1080, 1, 6),
    (1921, 1081, 3, 7),
    (3840, 2160, 1, 8),
    (12000, 100, 1, 11),      # a 12K-wide row: one level-1 row per band, > 64 KB of LDS requested
]


@pytest.mark.parametrize("w,h,ch,seed", CASES)
def test_pair_path_pyramids(mdx, oracle, w, h, ch, seed):
    a, b = frames(w, h, ch, seed)
    with mdx.Context(0, w, h, 1) as c:
        c.flow_warp_diff(a, b)
        c.sync()
        g1, g2 = oracle.to_gray(a), oracle.to_gray(b)
        check(mdx, c, oracle, [g1], [(2, [g1]), (3, [g2])], 1)


@pytest.mark.parametrize("w,h,ch,seed", [(333, 241, 1, 9), (1920, 1080, 3, 10)])
def test_trajectory_path_pyramids(mdx, oracle, w, h, ch, seed):
    a, b = frames(w, h, ch, seed)
    with mdx.Context(0, w, h, 1) as c:
        c.flow_trajectory([a, b])
        c.sync()
        g1, g2 = oracle.to_gray(a), oracle.to_gray(b)
        check(mdx, c, oracle, [g1], [(2, [g1]), (3, [g2])], 1)


@pytest.mark.parametrize("w,h,ch,B", [(640, 480, 3, 3), (1920, 1080, 1, 2)])
def test_batch_path_pyramids(mdx, oracle, w, h, ch, B):
    """Batched device entry: one k_front launch per frame side over B pairs (pair index in the grid)."""
    pairs = [frames(w, h, ch, 100 + i) for i in range(B)]
    fmt = mdx.FMT_GRAY8 if ch == 1 else mdx.FMT_RGB8
    fb = w * h * ch
    with mdx.Context(0, w, h, B) as c:
        d1, d2 = c.dev_alloc(fb * B), c.dev_alloc(fb * B)
        try:
            c.h2d(d1, np.stack([p[0] for p in pairs]))
            c.h2d(d2, np.stack([p[1] for p in pairs]))
            c.flow_warp_diff_batch_dev(B, d1, d2, w, h, w * ch, fb, fmt)
            c.sync()
            g1 = [oracle.to_gray(p[0]) for p in pairs]
            g2 = [oracle.to_gray(p[1]) for p in pairs]
            check(mdx, c, oracle, g1, [(2, g1), (3, g2)], B)
        finally:
            c.dev_free(d1)
            c.dev_free(d2)
