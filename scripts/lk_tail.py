"""Wave-occupancy profile of the persistent LK iteration kernel (GPU box, debug mode).

Runs the bench workload (1080p, 32 pairs of 4 distinct synthetic pairs) with MDX_LK_DEBUG=1, reads
every persistent wave's {start, end} s_memrealtime stamps per level (k_lk_iter writes them in debug
mode only) and prints, per level, the launch span and how long the chip ran with fewer waves:
the tail that level-major launches leave idle.
Usage (GPU box): MDX_LK_DEBUG=1 python scripts/lk_tail.py
"""
import ctypes as C
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np

import motion_detection_amd as m

K_MAX_LEVELS, STAMP_OFF, WAVES = 8, 8 * 64 + 64, 16384


def main():
    assert os.environ.get("MDX_LK_DEBUG") == "1", "run with MDX_LK_DEBUG=1"
    w, h, B = 1920, 1080, 32
    uniq = [m.synth_pair(20141105 + i, w, h, 1) for i in range(4)]
    g1 = np.stack([uniq[i % 4][0] for i in range(B)]); g2 = np.stack([uniq[i % 4][1] for i in range(B)])
    n = m.grid_count(w, h, 10)
    with m.Context(0, w, h, B, pixel_step=10, min_vector_size=1.0) as c:
        b1, b2 = c.dev_alloc(g1.nbytes), c.dev_alloc(g2.nbytes)
        c.h2d(b1, g1); c.h2d(b2, g2)
        for _ in range(3):
            c.flow_warp_diff_batch_dev(B, b1, b2, w, h, w, w * h, m.FMT_GRAY8)
        c.sync()
        nlev = 5
        total = (n * nlev * B + STAMP_OFF + K_MAX_LEVELS * WAVES) * 4
        buf = np.zeros(total, np.uint32)
        rc = m.lib().mdx_debug_copy(c._h, 1, buf.ctypes.data_as(C.c_void_p), buf.nbytes)
        assert rc == 0, rc
        c.dev_free(b1); c.dev_free(b2)
    st = buf[(n * nlev * B + STAMP_OFF) * 4:].reshape(K_MAX_LEVELS, WAVES, 4).astype(np.uint64)
    t0 = st[..., 0] | (st[..., 1] << np.uint64(32))
    t1 = st[..., 2] | (st[..., 3] << np.uint64(32))
    # all levels together (with MDX_LK_FLOW the launches overlap): summed wave lifetimes against
    # the resident capacity over the whole LK span
    ok_all = t1[:nlev] > 0
    s_all, e_all = t0[:nlev][ok_all].astype(np.int64), t1[:nlev][ok_all].astype(np.int64)
    if len(s_all):
        span_all = (e_all.max() - s_all.min()) * 10
        # k_lk_iter's resident capacity on MI355X: 256 CUs x 4 SIMDs x 4 waves (<= 128 VGPRs)
        cap = 4096
        use = ((e_all - s_all) * 10).sum() / (cap * span_all)
        print(f"all levels: span {span_all / 1e3:.0f} us, wave-time / ({cap} resident waves x span) {use:.3f}")
    for L in range(nlev - 1, -1, -1):
        ok = t1[L] > 0
        s, e = t0[L][ok].astype(np.int64), t1[L][ok].astype(np.int64)
        if not len(s):
            continue
        base = s.min()
        s, e = (s - base) * 10, (e - base) * 10                      # ns (100 MHz)
        span = e.max()
        ends = np.sort(e)
        nw = len(e)
        # time from when 10% / 50% / 90% of the waves have exited to the last exit
        q = {f: span - ends[int(f * nw) - 1] for f in (0.1, 0.5, 0.9)}
        busy = (e - s).sum() / (nw * span)
        print(f"level {L}: waves {nw}, span {span / 1e3:.0f} us, wave-time/(waves*span) {busy:.3f}, "
              f"after 10%/50%/90% exited: {q[0.1] / 1e3:.0f}/{q[0.5] / 1e3:.0f}/{q[0.9] / 1e3:.0f} us")
        # per XCD (blocks are dealt round-robin: wave index & 7): first and last exit, and its
        # waves' summed lifetime against waves x span -- imbalance between the XCDs' queue ranges
        # shows as a spread of the last exits
        idx = np.nonzero(ok)[0]
        xs = []
        for x in range(8):
            sel = (idx & 7) == x
            if sel.any():
                xs.append(f"{x}:{e[sel].min() / 1e3:.0f}-{e[sel].max() / 1e3:.0f}")
        print("    per-XCD first-last exit (us): " + " ".join(xs))


if __name__ == "__main__":
    main()
