"""The live chain's resident frame ring (include/mdx.h mdx_ring_*): the node's raw_images_ deque
(reference ros/src/motion_detection_node.cpp:248-261, re-converted and re-pyramided on every
callback at :266-287) kept in HBM, one upload and one pyramid per frame.

GPU: frames pushed one at a time; after every push that leaves >= 2 frames in the ring,
mdx_ring_trajectory equals the oracle's calculateOpticalFlowTrajectory over exactly those frames
(bit for bit: trajectories as float32 bits, lengths, start points, Vec4d, num_vectors), including a
ring that shrinks and grows (the deque's size follows trajectory_size = 2*num_motions+1, re-read
every frame at :239-241) and a frame-size change.  CPU: argument checks of the entry points.
"""
import numpy as np
import pytest

from traj_seq import sequence


def _compare(res, ref, label):
    assert res.num_vectors == ref["num_vectors"], label
    np.testing.assert_array_equal(res.traj_len, ref["traj_len"], err_msg=label)
    for i in range(len(res.traj_len)):
        k = int(ref["traj_len"][i])
        assert np.array_equal(res.traj[i, :k].view(np.uint32), ref["traj"][i, :k].view(np.uint32)), (label, i)
    np.testing.assert_array_equal(res.start_pts.view(np.uint32), ref["start_pts"].view(np.uint32), err_msg=label)
    np.testing.assert_array_equal(res.vectors.view(np.uint64), ref["vectors"].view(np.uint64), err_msg=label)


def deque_sizes(keeps):
    """The reference deque's size after each push (node.cpp:248-261): grow while below the wanted
    trajectory size, else push + pop (so a smaller trajectory size never shrinks it)."""
    n, out = 0, []
    for ts in keeps:
        n = n + 1 if n < ts else n
        out.append(n)
    return out


def test_deque_sizes_follow_the_reference():
    assert deque_sizes([5] * 8) == [1, 2, 3, 4, 5, 5, 5, 5]
    assert deque_sizes([5, 5, 5, 5, 5, 3, 3, 7, 7]) == [1, 2, 3, 4, 5, 5, 5, 6, 7]


def test_ring_rejects_bad_arguments(mdx):
    """CPU: argument checks run before any device work (no context needed for a null one)."""
    L = mdx.lib()
    assert L.mdx_ring_push(None, None, 4, 4, 4, 0, 1) < 0
    assert L.mdx_ring_trajectory(None, None, None, None, None, None) < 0
    assert L.mdx_ring_reset(None) < 0


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,ch,keeps", [
    (320, 240, 3, [5] * 8),                              # the node's default ring, 8 frames one at a time
    (640, 480, 1, [5, 5, 5, 5, 5, 3, 3, 7, 7, 7]),        # num_motions changed on the fly
])
def test_ring_matches_oracle_frame_by_frame(mdx, ctx, oracle, w, h, ch, keeps):
    frames = sequence(mdx, oracle, w, h, len(keeps), seed=41 + ch, channels=ch)
    sizes = deque_sizes(keeps)
    ctx.ring_reset()
    for k, (f, n) in enumerate(zip(frames, sizes)):
        assert ctx.ring_push(f, n) == n
        if n < 2:
            continue
        ring = frames[k + 1 - n:k + 1]
        res = ctx.ring_trajectory(w, h, n)
        ref = oracle.flow_trajectory(ring, pixel_step=10, nthreads=8)
        _compare(res, ref, f"frame {k}, ring of {n}")
        if k == len(frames) - 1:     # the list entry on the same frames gives the same result
            _compare(ctx.flow_trajectory(ring), ref, "list entry")


@pytest.mark.gpu
def test_ring_restarts_on_a_new_frame_size(mdx, ctx, oracle):
    a = sequence(mdx, oracle, 320, 240, 3, seed=7, channels=1)
    b = sequence(mdx, oracle, 200, 150, 3, seed=8, channels=1)
    ctx.ring_reset()
    for f in a:
        ctx.ring_push(f, 5)
    assert ctx.ring_push(b[0], 5) == 1                    # another size: the ring starts over
    for f in b[1:]:
        ctx.ring_push(f, 5)
    _compare(ctx.ring_trajectory(200, 150, 3), oracle.flow_trajectory(b, pixel_step=10), "after resize")
    ctx.ring_reset()
    with pytest.raises(mdx.MdxError):
        ctx.ring_trajectory(200, 150, 2)                  # empty ring


@pytest.mark.gpu
def test_ring_pushes_in_flight(mdx, ctx, oracle):
    """Pushes are queued, not done, when mdx_ring_push returns (include/mdx.h): five pushes queued
    before one trajectory call, then frames pushed from one reused page-locked buffer, rewritten
    only after the call returns."""
    w, h = 640, 480
    frames = sequence(mdx, oracle, w, h, 7, seed=77, channels=3)
    ctx.ring_reset()
    for f in frames[:5]:
        ctx.ring_push(f, 5)
    _compare(ctx.ring_trajectory(w, h, 5), oracle.flow_trajectory(frames[:5], pixel_step=10, nthreads=8),
             "five pushes in flight")
    buf = mdx.host_empty(frames[0].shape)
    for k in (5, 6):
        buf[...] = frames[k]
        ctx.ring_push(buf, 5)
        _compare(ctx.ring_trajectory(w, h, 5),
                 oracle.flow_trajectory(frames[k - 4:k + 1], pixel_step=10, nthreads=8), f"pinned push {k}")


@pytest.mark.gpu
def test_pinned_views_keep_the_block_alive(mdx):
    """A plain-ndarray view of a page-locked array (np.asarray, .view(np.ndarray),
    np.ascontiguousarray as ring_push takes it) keeps the block alive after the PinnedArray itself
    is gone: numpy collapses a view's base chain to the lowest buffer object, which owns the block."""
    import gc
    a = mdx.host_empty((64, 64))
    views = [np.asarray(a), a.view(np.ndarray), np.ascontiguousarray(a)]
    del a
    gc.collect()
    for i, v in enumerate(views):
        v[...] = i + 1                                    # use after free if the block was released
        assert int(v.sum()) == (i + 1) * 64 * 64


@pytest.mark.gpu
@pytest.mark.parametrize("nimg", [5, 3])
def test_mapped_outputs_equal_copied_outputs(mdx, ctx, oracle, nimg):
    """Outputs in one page-locked block (trajectory_buffers(pinned=True), mdx_trajectory_layout) are
    written by the chained launch itself; pageable ones are copied back.  Both hold the same bits,
    entries past traj_len included (0), and match the oracle."""
    w, h = 320, 240
    frames = sequence(mdx, oracle, w, h, nimg, seed=77, channels=3)
    ctx.ring_reset()
    for f in frames:
        ctx.ring_push(f, nimg)
    mapped = ctx.ring_trajectory(w, h, nimg, out=ctx.trajectory_buffers(w, h, nimg, pinned=True))
    copied = ctx.ring_trajectory(w, h, nimg, out=ctx.trajectory_buffers(w, h, nimg, pinned=False))
    assert mapped.num_vectors == copied.num_vectors
    for a, b in [(mapped.traj, copied.traj), (mapped.traj_len, copied.traj_len), (mapped.start_pts, copied.start_pts),
                 (mapped.vectors, copied.vectors)]:
        assert a.tobytes() == b.tobytes()
    for i in range(len(mapped.traj_len)):
        assert not mapped.traj[i, int(mapped.traj_len[i]):].any()
    _compare(mapped, oracle.flow_trajectory(frames, pixel_step=10, nthreads=8), "mapped")
