"""GPU parity of the exact configuration bench.py times, and the failure paths around it.

The headline step (bench.py main, config C1) is mdx_flow_warp_diff_batch_dev over 32 resident
1920x1080 gray pairs with the reference constants and pixel_step 10, called back to back without a
host sync and with call pipelining on.  That configuration engages machinery no smaller case does:
five pyramid levels, the LK level dataflow (batch a multiple of 8 and >= 16, 20736 points = a
multiple of 16, so level l-1's groups wait per pair on level l's retire counters; 4 pairs per XCD
range), level 0 on k_lk_iter<8, 112>, and alternating pyramid halves.  Every output of every pair
is compared with the oracle (reference optical_flow_calculator.cpp:71-127: calcOpticalFlowPyrLK,
classification, getPerspectiveTransform, warpPerspective, absdiff, threshold).

Also here: a dataflow hand-off that gives up is recovered within the call (the level is recomputed
in sequence: bit-exact, MDX_OK, counted by mdx_lk_fallbacks), and a pipelined call whose frames come
from a producer on another stream is correct once the producer's event is passed with
mdx_input_ready.
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W, H, B, PS = 1920, 1080, 32, 10


def _pairs(mdx, seeds, w, h):
    return {s: mdx.synth_pair(s, w, h, 1, 16) for s in seeds}


def _oracle_refs(oracle, pairs):
    return {s: oracle.calculate_optical_flow(a, b, nthreads=16, pixel_step=PS, min_vector_size=1.0)
            for s, (a, b, _) in pairs.items()}


def _stack(pairs, slot_seeds):
    g1 = np.stack([pairs[s][0] for s in slot_seeds])
    g2 = np.stack([pairs[s][1] for s in slot_seeds])
    return g1, g2


def _alloc_out(c, n, w, h, batch, vectors):
    sizes = dict(np=batch * n * 8, st=batch * n, mask=batch * w * h, H=batch * 72, num=batch * 4)
    if vectors:
        sizes["vec"] = batch * n * 32
    return {k: c.dev_alloc(v) for k, v in sizes.items()}


def _read_out(c, o, n, w, h, batch):
    r = dict(np=np.empty((batch, n, 2), np.float32), st=np.empty((batch, n), np.uint8),
             mask=np.empty((batch, h, w), np.uint8), H=np.empty((batch, 9)), num=np.empty(batch, np.int32))
    if "vec" in o:
        r["vec"] = np.empty((batch, n, 4))
    for k, arr in r.items():
        c.d2h(arr, o[k])
    return r


def _check_slot(got, i, ref, label):
    assert got["num"][i] == ref["num_vectors"], label
    np.testing.assert_array_equal(got["st"][i], ref["status"], err_msg=label)
    bad = np.nonzero((got["np"][i].view(np.uint32) != ref["next_pts"].view(np.uint32)).any(axis=1))[0]
    assert bad.size == 0, f"{label}: {bad.size} LK points differ, first {bad[:5]}"
    np.testing.assert_array_equal(got["H"][i].view(np.uint64), ref["H"].ravel().view(np.uint64), err_msg=label)
    nbad = int((got["mask"][i] != ref["mask"]).sum())
    assert nbad == 0, f"{label}: {nbad} mask pixels differ"
    if "vec" in got:
        np.testing.assert_array_equal(got["vec"][i], ref["vectors"], err_msg=label)


def _call(c, batch, d1, d2, o, w, h):
    c.flow_warp_diff_batch_dev(batch, d1, d2, w, h, w, w * h, 0, d_next_pts=o["np"], d_status=o["st"],
                               d_vectors=o.get("vec", 0), d_mask=o["mask"], d_H=o["H"], d_num_vectors=o["num"])


@pytest.mark.parametrize("xcall", ["0", "1"])
def test_benchmarked_path_1080p_x32_pipelined(mdx, oracle, monkeypatch, xcall):
    """bench.py's timed step, twice back to back on different inputs (16 distinct pairs, 8 per call,
    each in 4 of the 32 slots), call pipelining on, one sync at the end: every pair's next_pts
    (float32 bits), status, H (float64 bits), mask and num_vectors -- and the Vec4d of the second
    call -- equal the oracle's.  xcall "1": the same with MDX_LK_XCALL=1 (read at mdx_create; off by
    default), whose consecutive calls alternate the LK streams and counter sets so that one call's
    level 0 overlaps the next call's coarse levels."""
    monkeypatch.setenv("MDX_LK_XCALL", xcall)
    seeds_a = [20141105 + i for i in range(8)]
    seeds_b = [20141205 + i for i in range(8)]
    pairs = _pairs(mdx, seeds_a + seeds_b, W, H)
    refs = _oracle_refs(oracle, pairs)
    slots_a = [seeds_a[i % 8] for i in range(B)]
    slots_b = [seeds_b[(3 * i + 1) % 8] for i in range(B)]      # another spread over the slots
    n = mdx.grid_count(W, H, PS)
    assert n % 16 == 0 and B % 8 == 0 and B >= 16               # the dataflow's conditions hold
    with mdx.Context(0, W, H, B, pixel_step=PS, min_vector_size=1.0, call_pipelining=1) as c:
        ins = []
        for slots in (slots_a, slots_b):
            g1, g2 = _stack(pairs, slots)
            d1, d2 = c.dev_alloc(g1.nbytes), c.dev_alloc(g2.nbytes)
            c.h2d(d1, g1)
            c.h2d(d2, g2)
            ins.append((d1, d2))
        outs = [_alloc_out(c, n, W, H, B, vectors=False), _alloc_out(c, n, W, H, B, vectors=True)]
        # a warm-up call into the second output set first, so that the two checked calls run with
        # the previous call still in flight (the bench's steady state)
        _call(c, B, *ins[1], outs[1], W, H)
        _call(c, B, *ins[0], outs[0], W, H)
        _call(c, B, *ins[1], outs[1], W, H)
        c.sync()                                                # also the hand-off timeout check
        got = [_read_out(c, o, n, W, H, B) for o in outs]
        for o in outs:
            for p in o.values():
                c.dev_free(p)
        for d1, d2 in ins:
            c.dev_free(d1)
            c.dev_free(d2)
    for j, slots in enumerate((slots_a, slots_b)):
        for i, s in enumerate(slots):
            _check_slot(got[j], i, refs[s], f"call {j} slot {i} seed {s}")


def _small_batch(mdx, w=320, h=240, batch=16, seed0=900):
    pairs = _pairs(mdx, [seed0 + i for i in range(batch)], w, h)
    slots = [seed0 + i for i in range(batch)]
    return pairs, slots


@pytest.mark.parametrize("spin", ["-1", "2"])
def test_dataflow_fallback_is_bit_exact(mdx, oracle, monkeypatch, spin):
    """The benchmarked configuration (1080p x 32, call pipelining on, two calls in flight) with the
    dataflow's waits forced to give up: MDX_LK_SPIN_MAX=-1 (read at mdx_create) makes every wait and
    gate give up at once, as when the coarser level's launch is never dispatched beside the finer
    one (a preempted, shared or kernel-serializing device); 2 polls makes some give up and others
    not.  Each abandoned level is recomputed in sequence within the same call (launch_lk_v2), so
    the sync reports MDX_OK and every output is bit-exact against the oracle; the fallback counts
    say what happened (for -1: every level below the coarsest recomputed, in every call)."""
    monkeypatch.setenv("MDX_LK_SPIN_MAX", spin)
    seeds_a = [20141105 + i for i in range(8)]
    seeds_b = [20141305 + i for i in range(8)]
    pairs = _pairs(mdx, seeds_a + seeds_b, W, H)
    refs = _oracle_refs(oracle, pairs)
    slots_a = [seeds_a[i % 8] for i in range(B)]
    slots_b = [seeds_b[(5 * i + 3) % 8] for i in range(B)]
    n = mdx.grid_count(W, H, PS)
    with mdx.Context(0, W, H, B, pixel_step=PS, min_vector_size=1.0, call_pipelining=1) as c:
        ins = []
        for slots in (slots_a, slots_b):
            g1, g2 = _stack(pairs, slots)
            d1, d2 = c.dev_alloc(g1.nbytes), c.dev_alloc(g2.nbytes)
            c.h2d(d1, g1)
            c.h2d(d2, g2)
            ins.append((d1, d2))
        outs = [_alloc_out(c, n, W, H, B, vectors=True), _alloc_out(c, n, W, H, B, vectors=True)]
        _call(c, B, *ins[0], outs[0], W, H)
        _call(c, B, *ins[1], outs[1], W, H)
        c.sync()                                                # MDX_OK: no exception
        fb = c.lk_fallbacks()
        got = [_read_out(c, o, n, W, H, B) for o in outs]
        for o in outs:
            for p in o.values():
                c.dev_free(p)
        for d1, d2 in ins:
            c.dev_free(d1)
            c.dev_free(d2)
    print("fallbacks:", fb)
    if spin == "-1":
        nlev = 5                                                # 1080p: levels 0..4
        assert fb["group_giveups"] > 0 and fb["gate_giveups"] == 2 * (nlev - 1)
        assert fb["levels_recomputed"] == 2 * (nlev - 1)
    for j, slots in enumerate((slots_a, slots_b)):
        for i, s in enumerate(slots):
            _check_slot(got[j], i, refs[s], f"spin {spin} call {j} slot {i} seed {s}")


@pytest.mark.parametrize("mode,spin,w,h,batch", [("1", None, 1920, 1080, 1), ("1", None, 640, 480, 4),
                                                  ("2", None, 1920, 1080, 16), ("1", "-1", 640, 480, 4)])
def test_per_point_dataflow_bit_exact(mdx, oracle, monkeypatch, mode, spin, w, h, batch):
    """The opt-in per-point level dataflow (MDX_LK_PFLOW=1: batches the per-pair form does not take;
    2: every batch): a group waits only for its own points' coarser-level results, stamped with the
    call's epoch.  Two calls back to back (epochs 1 and 2, flags not cleared in between), pipelined;
    with MDX_LK_SPIN_MAX=-1 every wait gives up and the levels are recomputed.  Bit-exact."""
    monkeypatch.setenv("MDX_LK_PFLOW", mode)
    if spin:
        monkeypatch.setenv("MDX_LK_SPIN_MAX", spin)
    seeds = [31000 + i for i in range(min(batch, 4))]
    pairs = _pairs(mdx, seeds, w, h)
    refs = _oracle_refs(oracle, pairs)
    slots = [seeds[i % len(seeds)] for i in range(batch)]
    n = mdx.grid_count(w, h, PS)
    with mdx.Context(0, w, h, batch, pixel_step=PS, min_vector_size=1.0, call_pipelining=1) as c:
        g1, g2 = _stack(pairs, slots)
        d1, d2 = c.dev_alloc(g1.nbytes), c.dev_alloc(g2.nbytes)
        c.h2d(d1, g1)
        c.h2d(d2, g2)
        outs = [_alloc_out(c, n, w, h, batch, vectors=True) for _ in range(2)]
        for o in outs:
            _call(c, batch, d1, d2, o, w, h)
        c.sync()
        fb = c.lk_fallbacks()
        got = [_read_out(c, o, n, w, h, batch) for o in outs]
        for o in outs:
            for p in o.values():
                c.dev_free(p)
        c.dev_free(d1)
        c.dev_free(d2)
    if spin:
        assert fb["levels_recomputed"] > 0
    for j in range(2):
        for i, sd in enumerate(slots):
            _check_slot(got[j], i, refs[sd], f"pflow {mode} call {j} slot {i}")


def test_default_run_fallbacks_are_recovered(mdx, monkeypatch):
    """With the default wait bound the fallback counters are statistics, not errors: on an idle
    device they stay 0 (the bench reports them per run), while on a shared, preempted or
    profiler-serialized device a wait may give up -- then every give-up must have been followed by
    a recompute within the same call (mdx_sync would otherwise return MDX_EHIP)."""
    monkeypatch.delenv("MDX_LK_SPIN_MAX", raising=False)
    w, h, batch = 640, 480, 16
    pairs, slots = _small_batch(mdx, w, h, batch, seed0=990)
    n = mdx.grid_count(w, h, PS)
    with mdx.Context(0, w, h, batch, pixel_step=PS, min_vector_size=1.0, call_pipelining=1) as c:
        g1, g2 = _stack(pairs, slots)
        d1, d2 = c.dev_alloc(g1.nbytes), c.dev_alloc(g2.nbytes)
        c.h2d(d1, g1)
        c.h2d(d2, g2)
        o = _alloc_out(c, n, w, h, batch, vectors=False)
        for _ in range(4):
            _call(c, batch, d1, d2, o, w, h)
        c.sync()
        fb = c.lk_fallbacks()
        for p in list(o.values()) + [d1, d2]:
            c.dev_free(p)
    print("lk_fallbacks", fb)
    if fb["group_giveups"] + fb["gate_giveups"] > 0:
        assert fb["levels_recomputed"] > 0, fb
    else:
        assert fb["levels_recomputed"] == 0, fb


def _hip():
    """The HIP runtime libmdx.so is linked against (already loaded: dlopen returns it)."""
    L = C.CDLL("libamdhip64.so")
    vp = C.c_void_p
    L.hipStreamCreate.argtypes = [C.POINTER(vp)]
    L.hipEventCreate.argtypes = [C.POINTER(vp)]
    L.hipHostMalloc.argtypes = [C.POINTER(vp), C.c_size_t, C.c_uint]
    L.hipMemcpyAsync.argtypes = [vp, vp, C.c_size_t, C.c_int, vp]
    L.hipEventRecord.argtypes = [vp, vp]
    L.hipStreamSynchronize.argtypes = [vp]
    L.hipStreamDestroy.argtypes = [vp]
    L.hipEventDestroy.argtypes = [vp]
    L.hipHostFree.argtypes = [vp]
    L.hipMalloc.argtypes = [C.POINTER(vp), C.c_size_t]
    L.hipFree.argtypes = [vp]
    return L


def test_input_ready_event_from_producer_stream(mdx, oracle):
    """Zero-copy producer on its own stream: a large copy queued first keeps that stream busy, the
    frames follow, an event is recorded behind them and handed over with mdx_input_ready.  The
    pipelined call (its front end on the context's second stream, not behind the context stream)
    waits for it: results bit-exact.  The device buffers hold zeros before the producer writes, so
    a front end that ran early would have read the wrong frames."""
    hip = _hip()
    w, h, batch = 640, 480, 16
    pairs, slots = _small_batch(mdx, w, h, batch, seed0=980)
    refs = _oracle_refs(oracle, pairs)
    n = mdx.grid_count(w, h, PS)
    g1, g2 = _stack(pairs, slots)
    vp = C.c_void_p
    st, ev, host, big_h, big_d = vp(), vp(), vp(), vp(), vp()
    BIG = 256 << 20
    assert hip.hipStreamCreate(C.byref(st)) == 0
    assert hip.hipEventCreate(C.byref(ev)) == 0
    assert hip.hipHostMalloc(C.byref(host), 2 * g1.nbytes, 0) == 0
    assert hip.hipHostMalloc(C.byref(big_h), BIG, 0) == 0
    try:
        hb = np.ctypeslib.as_array(C.cast(host, C.POINTER(C.c_uint8)), shape=(2 * g1.nbytes,))
        hb[:g1.nbytes] = g1.ravel()
        hb[g1.nbytes:] = g2.ravel()
        with mdx.Context(0, w, h, batch, pixel_step=PS, min_vector_size=1.0, call_pipelining=1) as c:
            assert hip.hipMalloc(C.byref(big_d), BIG) == 0
            d1, d2 = c.dev_alloc(g1.nbytes), c.dev_alloc(g2.nbytes)
            z = np.zeros(g1.nbytes, np.uint8)
            c.h2d(d1, z)
            c.h2d(d2, z)
            o = _alloc_out(c, n, w, h, batch, vectors=True)
            assert hip.hipMemcpyAsync(big_d, big_h, BIG, 1, st) == 0          # keeps the producer busy
            assert hip.hipMemcpyAsync(vp(d1), host, g1.nbytes, 1, st) == 0
            assert hip.hipMemcpyAsync(vp(d2), vp(host.value + g1.nbytes), g2.nbytes, 1, st) == 0
            assert hip.hipEventRecord(ev, st) == 0
            c.input_ready(ev.value)
            _call(c, batch, d1, d2, o, w, h)
            c.sync()
            got = _read_out(c, o, n, w, h, batch)
            assert hip.hipStreamSynchronize(st) == 0
            for p in list(o.values()) + [d1, d2]:
                c.dev_free(p)
            hip.hipFree(big_d)
    finally:
        hip.hipHostFree(host)
        hip.hipHostFree(big_h)
        hip.hipEventDestroy(ev)
        hip.hipStreamDestroy(st)
    for i, s in enumerate(slots):
        _check_slot(got, i, refs[s], f"slot {i}")
