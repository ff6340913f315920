#!/usr/bin/env python
"""Benchmark of the flow + egomotion-warp + frame-difference hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 1080p|4k|640]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A *step* = one pass of the whole reference path (gray+pad, pyramids, Scharr, pyramidal LK,
first-4 perspective fit, back-warp + absdiff + threshold) over a batch of B synthetic frame
pairs already resident in HBM.  Each rank is one independent camera-stream shard on its own
GPU (LOCAL_RANK) with its own seeds: no data-path collective; torch.distributed (gloo) is used
only for the barrier and the max-over-ranks timing.  value = pixels of frame 2 processed by
all ranks / max-over-ranks wall time, in Mpixels/s (weak scaling).

Also reported, for the north-star kernel (fused warp+diff, rows A8-A10) on 4K pairs with the
generator's true homography: achieved algorithmic HBM GB/s vs the 8 TB/s peak ("roofline"),
and the CPU oracle (C restatement of the reference path) timed on this host ("cpu_baseline").
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import motion_detection_amd as mdx  # noqa: E402  (loads libmdx.so before torch)

METRIC = "Mpixels/s (flow+warp+diff) at 1080p & 4K; % HBM roofline, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md chip table)
CONFIGS = {"640": (640, 480), "1080p": (1920, 1080), "4k": (3840, 2160), "8k": (7680, 4320)}
SEED0 = 20141105


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class Dist:
    """Rank bookkeeping; torch.distributed (gloo) only when WORLD_SIZE > 1."""

    def __init__(self):
        self.rank = int(os.environ.get("RANK", 0))
        self.world = int(os.environ.get("WORLD_SIZE", 1))
        self.local_rank = int(os.environ.get("LOCAL_RANK", 0))
        self.dist = None
        if self.world > 1:
            import torch
            import torch.distributed as dist
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo", rank=self.rank, world_size=self.world)
            self.torch, self.dist = torch, dist

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def max(self, v: float) -> float:
        if self.dist is None:
            return v
        t = self.torch.tensor([v], dtype=self.torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def sum(self, v: float) -> float:
        if self.dist is None:
            return v
        t = self.torch.tensor([v], dtype=self.torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())

    def allgather_bytes(self, b: bytes) -> list:
        """Every rank's equal-length byte string, in rank order (the row-tiled path's record
        exchange: 96 B per rank, host-side over gloo)."""
        if self.dist is None:
            return [b]
        t = self.torch.frombuffer(bytearray(b), dtype=self.torch.uint8)
        out = [self.torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(out, t)
        return [bytes(o.numpy().tobytes()) for o in out]

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()


def throughput(D: Dist, units_local: float, seconds_local: float):
    """Whole-job rate: units processed by all ranks / max-over-ranks wall time (the slowest
    shard bounds the job).  Returns (rate, max_seconds)."""
    t = D.max(seconds_local)
    return D.sum(units_local) / t, t


def make_batch(w: int, h: int, batch: int, unique: int, seed0: int, threads: int):
    """`unique` distinct synthetic pairs replicated to `batch` slots (distinct HBM addresses,
    so the working set still exceeds the 256 MB Infinity Cache)."""
    uniq = [mdx.synth_pair(seed0 + i, w, h, 1, threads) for i in range(unique)]
    g1 = np.empty((batch, h, w), np.uint8)
    g2 = np.empty((batch, h, w), np.uint8)
    for i in range(batch):
        g1[i], g2[i] = uniq[i % unique][0], uniq[i % unique][1]
    Ht = uniq[0][2]
    return g1, g2, Ht, uniq


def host_cores() -> dict:
    """What this host offers: nproc (the CPUs this process may run on), the cgroup CPU quota, which
    on a shared GPU box can be far smaller than nproc (256 CPUs visible, 16 granted), and the CPUs
    actually available = min(nproc, quota): the thread count the CPU baseline uses and reports."""
    nproc = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    avail = nproc if quota is None else max(1, min(nproc, int(quota)))
    return {"nproc": nproc, "cgroup_cpu_quota": quota, "available": avail}


def stamped_pmc(path: str, key: str, expect: str):
    """A counter summary under profiles/ only when it was measured on the sources of the loaded
    library: its src_sha256 (the bench line's build stamp in the profiled run) must equal this
    build's, and its config string must match.  Otherwise None (the line then carries null)."""
    if not os.path.exists(path):
        return None
    with open(path) as f:
        pj = json.load(f)
    if pj.get("config") != expect or pj.get("src_sha256") != mdx._lib.build_info().get("src_sha256"):
        return None
    return pj


def cpu_baseline(uniq, w, h, seconds: float, threads: int, simd: bool = True):
    """The C oracle on this host: whole reference path per pair, `threads` threads over LK
    points / warp rows (like OpenCV's parallel_for_).  simd: the LK sums and the warp's bilinear
    through the SSE2 restatement (oracle/mdx_oracle_sse2.c, OpenCV 2.4's own x86 lane order, same
    results), which is what the reference's x86 OpenCV build runs; otherwise the scalar loops.
    Bounded sample: pairs are processed until `seconds` of wall time have elapsed (at least one)."""
    from oracle import pyoracle
    pyoracle.build()
    n, t0 = 0, time.perf_counter()
    while True:
        a, b, _ = uniq[n % len(uniq)]
        pyoracle.calculate_optical_flow(a, b, nthreads=threads, pixel_step=10, min_vector_size=1.0, simd=simd)
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    what = ("SSE2-intrinsics restatement of the OpenCV 2.4 x86 path (oracle/mdx_oracle_sse2.c: LK window/iteration "
            "sums and warp bilinear in 4-lane vectors; pyramids, Scharr and fit scalar, <3% of the time)"
            if simd else "scalar C restatement of the OpenCV 2.4 path (oracle/mdx_oracle.c)")
    return dict(value=round(n * w * h / 1e6 / el, 3), unit="Mpixels/s", cores=threads,
                kind="port-sse2" if simd else "port",
                sample=f"{n} x {w}x{h} gray pairs, full reference path ({what}, {threads} thread(s) over LK points / "
                       f"warp rows), {el:.1f} s wall")


def check_outputs(uniq, outs, B, w, h, ps, threads):
    """Untimed checker (test infrastructure, like cpu_baseline): the oracle's results for the
    `unique` distinct pairs, compared bit for bit with every one of the B slots of the last timed
    step (slot i holds pair i % unique): next_pts (float32 bits), status, Vec4d (float64 bits), H
    (float64 bits), mask and num_vectors.  Returns the counts; a mismatch is reported in the line, never hidden."""
    from oracle import pyoracle
    pyoracle.build()
    refs = [pyoracle.calculate_optical_flow(a, b, nthreads=threads, pixel_step=ps, min_vector_size=1.0, simd=True)
            for a, b, _ in uniq]
    bad = []
    for i in range(B):
        r = refs[i % len(refs)]
        diffs = []
        if int(outs["num"][i]) != r["num_vectors"]:
            diffs.append("num_vectors")
        if not np.array_equal(outs["st"][i], r["status"]):
            diffs.append("status")
        if not np.array_equal(outs["np"][i].view(np.uint32), r["next_pts"].view(np.uint32)):
            diffs.append("next_pts")
        if not np.array_equal(outs["vec"][i].view(np.uint64), np.asarray(r["vectors"], np.float64).reshape(-1, 4).view(np.uint64)):
            diffs.append("vectors")
        if not np.array_equal(outs["H"][i].view(np.uint64), r["H"].ravel().view(np.uint64)):
            diffs.append("H")
        if not np.array_equal(outs["mask"][i], r["mask"]):
            diffs.append("mask")
        if diffs:
            bad.append({"slot": i, "differs": diffs})
    return dict(checked_pairs=B, distinct_pairs=len(refs), mismatched_pairs=len(bad), mismatches=bad[:8],
                compared="next_pts bits, status, Vec4d bits, H bits, mask, num_vectors vs oracle/ (untimed)")


REHEARSE = False   # --rehearse: ranks beyond the visible devices may share device 0


VALU_PEAK_WAVE_INSTR = 1024 * 2.4e9 / 4   # 1024 SIMDs x 2.4 GHz, one wave64 VALU instruction per 4 cycles (the
                                          # issue cost of one wave's stream, measured on this op mix)
VALU_PEAK_WAVE_INSTR_2CYC = 1024 * 2.4e9 / 2   # the SIMD's 2-cycle wave64 rate (MI355X_MICROARCH.md:54, :473)
LK_VALU_PER_ELEM_ITER = 5   # minimal per window element and Newton iteration: 2 v_dot2 (bilinear J, folded I),
                            # 1 cvt, 1 v_pk_mul_f32 + 1 v_pk_add_f32 (b1, b2 products rounded before the add)
LK_VALU_PER_ELEM_A = 2      # minimal per element of the gradient sums: 1 v_pk_fma_f32 + 1 v_fma_f32 (A11/A22, A12)


def lk_levels(w: int, h: int, max_level: int = 5, win: int = 40) -> int:
    """Pyramid levels the LK runs (buildOpticalFlowPyramid stops when a side would be <= win)."""
    L = 0
    while L < max_level and (w + 1) // 2 > win and (h + 1) // 2 > win:
        w, h, L = (w + 1) // 2, (h + 1) // 2, L + 1
    return L + 1


def lk_work(dev: int, w: int, h: int, ps: int, uniq) -> dict:
    """Per-point Newton iterations of the pyramidal LK on the bench's distinct pairs, from the
    kernel's own per-(level, point) trace (MDX_LK_DEBUG context, untimed).  Returns the
    algorithmic VALU lane-instructions per pair: 1600 window elements x (LK_VALU_PER_ELEM_A per
    tracked (level, point) + LK_VALU_PER_ELEM_ITER per executed iteration)."""
    import ctypes as C
    os.environ["MDX_LK_DEBUG"] = "1"
    try:
        ctx = mdx.Context(dev, w, h, 1, pixel_step=ps, min_vector_size=1.0)
    finally:
        del os.environ["MDX_LK_DEBUG"]
    n, nl = mdx.grid_count(w, h, ps), lk_levels(w, h)
    its, trk = [], []
    for a, b, _ in uniq:
        ctx.flow_warp_diff(a, b)
        buf = np.zeros((nl, n, 4), np.float32)
        rc = mdx.lib().mdx_debug_copy(ctx._h, 1, buf.ctypes.data_as(C.c_void_p), buf.nbytes)
        if rc != 0:
            raise mdx.MdxError(f"mdx_debug_copy rc {rc}")
        it = buf[..., 2]
        its.append(float(it.sum()))
        trk.append(float((it >= 1).sum()))
    ctx.close()
    it_pair, trk_pair = float(np.mean(its)), float(np.mean(trk))
    lanes = 1600.0 * (LK_VALU_PER_ELEM_A * trk_pair + LK_VALU_PER_ELEM_ITER * it_pair)
    return dict(iterations_per_pair=round(it_pair, 1), iterations_per_point=round(it_pair / n, 3),
                tracked_level_points_per_pair=round(trk_pair, 1), valu_lane_instr_per_pair=lanes, levels=nl)


def open_ctx(D: Dist, w: int, h: int, batch: int, **params):
    """One context on this rank's GPU (LOCAL_RANK).  A rank whose device is not visible is an
    error (exit 3) unless --rehearse is given: then it shares device 0, and the JSON line's n_gpus
    counts the distinct devices actually used, never the ranks."""
    try:
        return mdx.Context(D.local_rank, w, h, batch, **params)
    except mdx.MdxError as e:
        if "out of range" not in str(e) and "invalid device" not in str(e).lower():
            raise
        if not REHEARSE:
            log(f"rank {D.rank}: device {D.local_rank} is not visible ({e}); refusing to share a GPU "
                f"(pass --rehearse to rehearse {D.world} ranks on fewer devices)")
            sys.exit(3)
        log(f"rank {D.rank}: device {D.local_rank} not visible, sharing device 0 (--rehearse)")
        return mdx.Context(0, w, h, batch, **params)


def device_summary(records):
    """records: one (rank, device, pci_bus_id) per rank.  Returns the JSON fields describing the
    devices used: n_gpus = number of DISTINCT physical devices (PCI ids), not ranks."""
    recs = sorted(records)
    pcis = [r[2] for r in recs]
    return {"n_gpus": len(set(pcis)), "ranks": len(recs),
            "devices": [{"rank": r[0], "device": r[1], "pci": r[2]} for r in recs]}


def gather_devices(D: Dist, ctx) -> dict:
    """Every rank's (rank, device id, PCI bus id), gathered over the host group."""
    rec = json.dumps([D.rank, ctx.device, ctx.device_pci()]).encode().ljust(128)
    parts = D.allgather_bytes(rec)
    return device_summary([tuple(json.loads(p.decode().strip())) for p in parts])


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` without a launcher: start N fresh worker processes of this script (one
    per GPU, RANK = LOCAL_RANK = i, WORLD_SIZE = N, gloo rendezvous on 127.0.0.1) and return the
    worst exit code.  The parent never touches the GPU and is never replaced (no exec)."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    # poll every child: as soon as one rank fails, end its siblings (they would otherwise sit in a
    # gloo collective waiting for it) and return that rank's code
    while True:
        rcs = [p.poll() for p in procs]
        bad = [rc for rc in rcs if rc not in (None, 0)]
        if bad:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=30)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            return bad[0]
        if all(rc == 0 for rc in rcs):
            return 0
        time.sleep(0.2)


def probe_ranks(D: Dist) -> None:
    """--probe-ranks: the launch plumbing alone (no GPU): every rank reports its env over gloo."""
    rec = json.dumps([D.rank, D.local_rank, D.world, os.getpid()]).encode().ljust(128)
    parts = [json.loads(p.decode().strip()) for p in D.allgather_bytes(rec)]
    if D.rank == 0:
        print(json.dumps({"probe": sorted(parts)}), flush=True)
    D.close()


def main_c4(args, D: Dist, threads: int):
    """Config C4: 8K RGB pairs row-tiled over the ranks.  `--bands K` splits the frame
    into K bands dealt round-robin to the ranks (K > ranks rehearses a K-GPU split on fewer GPUs).
    Per frame: each rank runs its bands' flow, the 96-byte band records are all-gathered (gloo,
    host side), then each rank fits (identically) and writes its bands' mask rows.
    `--inflight F` (default 2) keeps F consecutive frames in flight per GPU, each on its own context
    and HIP stream: one frame's band LK (a few thousand points, latency-bound, half the chip idle)
    overlaps the next frame's front end and LK.  A step is F frames; strong scaling: the frames are
    fixed, `value` = F x frame pixels / max-over-ranks step time."""
    from motion_detection_amd import rowtile
    w, h = CONFIGS[args.config] if args.config != "1080p" else CONFIGS["8k"]
    ps, fmt = 10, mdx.FMT_RGB8
    K = args.bands or D.world
    F = max(1, args.inflight)
    mine = list(range(D.rank, K, D.world))
    per_rank = -(-K // D.world)
    a, b, _ = mdx.synth_pair(SEED0 + 4, w, h, 3, threads)       # every rank: the same frame pair
    ctxs = [open_ctx(D, w, h, 1, pixel_step=ps, min_vector_size=1.0) for _ in range(F)]
    devs = gather_devices(D, ctxs[0])
    n = mdx.grid_count(w, h, ps)
    bufs = []
    for c in ctxs:
        d = {k: c.dev_alloc(sz) for k, sz in dict(i1=a.nbytes, i2=b.nbytes, np=n * 8, st=n, cand=per_rank * 96,
                                                 cands=K * 96, mask=w * h, num=4).items()}
        c.h2d(d["i1"], a)
        c.h2d(d["i2"], b)
        bufs.append(d)
    rows = [rowtile.band_rows(h, K, k) for k in range(K)]
    pad = bytes(96)
    t_ph = {"flow": 0.0, "exchange": 0.0, "fit_warp": 0.0}

    def exchange(c, d):
        rec = np.empty(per_rank * 96, np.uint8)
        c.d2h(rec, d["cand"])                                    # the stream is drained: a plain copy
        local = rec.tobytes()[:96 * len(mine)] + pad * (per_rank - len(mine))
        parts = D.allgather_bytes(local)
        allrec = bytearray(K * 96)
        for r, part in enumerate(parts):                         # rank r holds bands r, r + world, ...
            for j, k in enumerate(range(r, K, D.world)):
                allrec[96 * k:96 * (k + 1)] = part[96 * j:96 * (j + 1)]
        c.h2d(d["cands"], np.frombuffer(bytes(allrec), np.uint8))

    def step(timed=False):
        t0 = time.perf_counter()
        for c, d in zip(ctxs, bufs):                             # every in-flight frame's flow, async
            for j, k in enumerate(mine):
                c.band_flow_dev(d["i1"], d["i2"], w, h, w * 3, fmt, *rows[k], d["np"], d["st"], d["cand"] + 96 * j)
        t1 = time.perf_counter()
        tx = tw = 0.0
        for c, d in zip(ctxs, bufs):                             # then, frame by frame: records, fit, warp
            e0 = time.perf_counter()
            c.sync()                                             # this frame's flow (its stream) is done
            e1 = time.perf_counter()
            exchange(c, d)
            tw += e1 - e0
            tx += time.perf_counter() - e1
            for k in mine:
                c.band_fit_warp_dev(K, d["cands"], *rows[k], d["mask"] + rows[k][0] * w, 0, d["num"])
        for c in ctxs:
            c.sync()
        t3 = time.perf_counter()
        if timed:
            t_ph["flow"] += t1 - t0 + tw                         # launches + waits for the flow streams
            t_ph["exchange"] += tx                               # record d2h + all-gather + h2d only
            t_ph["fit_warp"] += t3 - t1 - tx - tw

    for _ in range(args.warmup):
        step()
    D.barrier()
    for c in ctxs:
        c.device_sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(timed=True)
    for c in ctxs:
        c.device_sync()
    D.barrier()
    el = time.perf_counter() - t0
    el_max = D.max(el)
    num = np.empty(1, np.int32)
    ctxs[0].d2h(num, bufs[0]["num"])
    # one band alone per in-flight frame (K bands on K GPUs: each GPU's share), timed here for the
    # rehearsal case: F frames of band mine[0], amortised per frame
    band_ms = None
    if K > D.world and mine:
        k = mine[0]
        reps = max(2, args.steps)
        for c in ctxs:
            c.device_sync()
        tb = time.perf_counter()
        for _ in range(reps):
            for c, d in zip(ctxs, bufs):
                c.band_flow_dev(d["i1"], d["i2"], w, h, w * 3, fmt, *rows[k], d["np"], d["st"], d["cand"])
            for c, d in zip(ctxs, bufs):
                c.band_fit_warp_dev(K, d["cands"], *rows[k], d["mask"] + rows[k][0] * w, 0, d["num"])
        for c in ctxs:
            c.device_sync()
        band_ms = (time.perf_counter() - tb) / (reps * F) * 1e3
    for c, d in zip(ctxs, bufs):
        for p in d.values():
            c.dev_free(p)
    out = {
        "metric": METRIC,
        "value": round(args.steps * F * w * h / el_max / 1e6, 2),
        "unit": "Mpixels/s",
        "n_gpus": devs["n_gpus"],
        "ranks": devs["ranks"],
        "devices": devs["devices"],
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el_max / args.steps * 1e3, 3),
        "ms_per_frame": round(el_max / (args.steps * F) * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (mdx_synth_pair, rgb8)",
        "config": {"workload": f"C4: {w}x{h} RGB pairs, {F} in flight per GPU, each row-tiled into {K} bands over "
                               f"{D.world} rank(s); per band LK + classify, one 96-B record all-gather, "
                               f"identical fit on every rank, band warp+absdiff+threshold",
                   "frame": f"{w}x{h}", "pixel_step": ps, "bands": K, "bands_per_rank": per_rank, "inflight": F,
                   "parallelism": f"row bands, {D.world} rank(s), record exchange over gloo (host)"},
        "phase_ms_per_step_rank0": {k: round(v / args.steps * 1e3, 3) for k, v in t_ph.items()},
        "one_band_ms": round(band_ms, 3) if band_ms else None,
        "num_vectors": int(num[0]),
        "lk_fallbacks": [c.lk_fallbacks() for c in ctxs],
        "roofline": None,
        "cpu_baseline": None,
    }
    if D.rank == 0:
        print(json.dumps(out), flush=True)
    for c in ctxs:
        c.close()
    D.close()


def live_leg(dev, w, h, threads, with_cpu=True, reps=5):
    """The node's live chain (node.cpp:241-348): calculateOpticalFlowTrajectory
    over 2*num_motions+1 = 5 rgb8 frames, then fitSubspace(num_motions 2, sigma 0.5) on the complete
    trajectories.  trajectory_ms is the median of 8 * reps steady-state callbacks of the node's path:
    the new frame pushed into the resident ring (H2D of one rgb8 frame + its pyramid) and the
    trajectory over the ring's 5 frames (D2H of the outputs included; page-locked host buffers, as
    the node keeps them); trajectory_list_ms is the host-list entry
    (mdx_flow_trajectory: all 5 frames uploaded and pyramided per call)."""
    import ctypes as C
    a, b, _ = mdx.synth_pair(SEED0 + 5, w, h, 3, threads)
    frames = [a, b, a, b, a]          # the generator's pair, back and forth: every pass tracks
    ctx = mdx.Context(dev, w, h, 4, pixel_step=10, min_vector_size=1.0)
    rng = mdx._lib.MdxRandState()
    mdx.lib().mdx_srand(C.byref(rng), SEED0)
    res = ctx.flow_trajectory(frames)
    traj = np.ascontiguousarray(np.array(res.trajectories, np.float32))
    ctx.fit_subspace(traj, 2, 0.5, rng)
    t0 = time.perf_counter()
    for _ in range(reps):
        res = ctx.flow_trajectory(frames)
    t1 = time.perf_counter()
    traj = np.ascontiguousarray(np.array(res.trajectories, np.float32))
    t2 = time.perf_counter()
    for _ in range(reps):
        sub = ctx.fit_subspace(traj, 2, 0.5, rng)
    t3 = time.perf_counter()
    # the node's callback on the resident ring: frames arrive one at a time, alternating a, b.  The
    # node keeps its rgb8 staging frame and its output arrays in page-locked memory, allocated once
    # (mdx_host_alloc), so the frame upload and the readback are DMA at link rate
    pinned = os.environ.get("MDX_BENCH_PAGEABLE", "0") == "0"     # (A/B: 1 = pageable host buffers)
    pa, pb = (mdx.host_empty(a.shape), mdx.host_empty(b.shape)) if pinned else (a.copy(), b.copy())
    pa[...] = a
    pb[...] = b
    pout = ctx.trajectory_buffers(w, h, 5, pinned=pinned)
    ctx.ring_reset()
    for k in range(5):
        ctx.ring_push(pa if k % 2 == 0 else pb, 5)
    rres = ctx.ring_trajectory(w, h, 5, out=pout)
    same = bool(np.array_equal(rres.traj.view(np.uint32), res.traj.view(np.uint32)) and
                rres.num_vectors == res.num_vectors)
    cb = []
    for k in range(8 * reps):        # an even count: the ring then holds a b a b a again
        t4 = time.perf_counter()
        ctx.ring_push(pb if k % 2 == 0 else pa, 5)
        rres = ctx.ring_trajectory(w, h, 5, out=pout)
        cb.append(time.perf_counter() - t4)
    ctx.close()
    out = dict(workload=f"5 x {w}x{h} rgb8 frames, pixel_step 10: node callback on the resident ring "
                        f"(mdx_ring_push + mdx_ring_trajectory) + mdx_fit_subspace (num_motions 2, sigma 0.5, "
                        f"50 hypotheses)",
               trajectory_ms=round(float(np.median(cb)) * 1e3, 3),
               trajectory_ms_mean=round(float(np.mean(cb)) * 1e3, 3), callbacks=len(cb),
               trajectory_list_ms=round((t1 - t0) / reps * 1e3, 3), fit_subspace_ms=round((t3 - t2) / reps * 1e3, 3),
               ring_equals_list=same,
               points=int(len(res.traj_len)), complete_trajectories=int(len(traj)),
               outliers=int(sub.is_outlier.sum()),
               includes="ring: H2D of the new frame + D2H of the outputs (page-locked host buffers); list: H2D of "
                        "all 5 frames (pageable)")
    if with_cpu:
        from oracle import pyoracle   # CPU baseline leg only (test infrastructure)
        c0 = time.perf_counter()
        r = pyoracle.flow_trajectory(frames, nthreads=threads, pixel_step=10)
        c1 = time.perf_counter()
        pyoracle.fit_subspace(np.ascontiguousarray(np.array(r["trajectories"], np.float32)), 2, 0.5,
                              pyoracle.rand_state(SEED0))
        c2 = time.perf_counter()
        out["cpu_oracle"] = dict(trajectory_ms=round((c1 - c0) * 1e3, 1), fit_subspace_ms=round((c2 - c1) * 1e3, 1),
                                 cores=threads, kind="port")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="1080p", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=0, help="pairs per step per GPU (default 32 @1080p)")
    ap.add_argument("--cold-idle", type=float, default=1.0,
                    help="roofline leg: idle seconds before the timed cold burst (reported as roofline.cold_burst)")
    ap.add_argument("--unique", type=int, default=32,
                    help="distinct synthetic pairs per rank (default 32: every slot of the 1080p batch its own "
                         "content, BASELINE.md §2)")
    ap.add_argument("--roofline-config", default="4k", choices=sorted(CONFIGS))
    ap.add_argument("--roofline-batch", type=int, default=32)
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--roofline-warmup", type=int, default=200,
                    help="untimed launches before each roofline leg's timed ones: after idle, a burst of warp "
                         "launches runs its first ~120 in a clock / power transient (profiles/r05_warp_transient.txt)")
    ap.add_argument("--roofline-h", default="both", choices=["both", "affine", "projective"],
                    help="roofline leg launches: the affine true H, the projective H, or both (profiling passes "
                         "take one kind at a time so per-launch counters and records stay per kind)")
    ap.add_argument("--only-roofline", action="store_true", help="profiling aid: only the warp+diff roofline leg")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="main CPU-baseline leg (all CPUs, SSE2); the 1-core and scalar legs take half")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_warp_diff.json"),
                    help="per-launch HBM traffic measured by rocprofv3 --pmc (scripts/profile.sh)")
    ap.add_argument("--workload", default="c1", choices=["c1", "c4"],
                    help="c1: batched 1080p stream shards (the metric's config); c4: 8K RGB row-tiled")
    ap.add_argument("--bands", type=int, default=0, help="c4: row bands (default: one per rank)")
    ap.add_argument("--inflight", type=int, default=2, help="c4: frames in flight per GPU (one context each)")
    ap.add_argument("--no-live", action="store_true", help="skip the node's live trajectory + RANSAC leg")
    ap.add_argument("--no-4k", action="store_true", help="skip the whole-path 4K leg (config C2)")
    ap.add_argument("--no-ransac", action="store_true", help="skip the MDX_FIT_RANSAC whole-path leg")
    ap.add_argument("--rehearse", action="store_true",
                    help="allow more ranks than visible GPUs (they share device 0; n_gpus counts distinct devices)")
    ap.add_argument("--no-lk-roofline", action="store_true", help="skip the LK iteration census (profiling runs)")
    ap.add_argument("--probe-ranks", action="store_true", help="launch plumbing only: ranks report over gloo, no GPU")
    ap.add_argument("--no-pipelining", action="store_true", help="time the main leg with call pipelining off")
    ap.add_argument("--no-parity", action="store_true", help="skip the untimed oracle check of the last step")
    args = ap.parse_args()
    global REHEARSE
    REHEARSE = args.rehearse

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))          # one fresh worker process per GPU
    D = Dist()
    if args.gpus != D.world:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE {D.world}; using WORLD_SIZE")
    if args.probe_ranks:
        return probe_ranks(D)
    # host threads for the synthetic generator (bounded: the GPU box's CPU share is 16)
    threads = max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))))
    if args.workload == "c4":
        return main_c4(args, D, threads)
    # Call pipelining (mdx_params.call_pipelining): a device-entry call's front end may
    # start beside the previous call's last LK level and fit/warp.  Its contract -- inputs already in
    # HBM when the call is made -- holds here (the synthetic pairs are uploaded once, before the timed
    # steps).  The line also reports the rate without it (value_unpipelined).  C4's band calls measured
    # 3% slower with it, so that workload leaves it off.
    pipe = 0 if args.no_pipelining else 1
    w, h = CONFIGS[args.config]
    B = args.batch or {"640": 128, "1080p": 32, "4k": 8, "8k": 2}[args.config]
    unique = max(1, min(args.unique, B))
    ps = 10

    g1, g2, Ht, uniq = make_batch(w, h, B if not args.only_roofline else 1, unique if not args.only_roofline else 1,
                                  SEED0 + 1000 * D.rank, threads)
    if args.only_roofline:
        B, unique = 1, 1
    ctx = open_ctx(D, w, h, B, pixel_step=ps, min_vector_size=1.0, call_pipelining=pipe)
    devs = gather_devices(D, ctx)
    n = mdx.grid_count(w, h, ps)
    d1, d2 = ctx.dev_alloc(g1.nbytes), ctx.dev_alloc(g2.nbytes)
    dout = {k: ctx.dev_alloc(sz) for k, sz in dict(np=B * n * 8, st=B * n, vec=B * n * 32, mask=B * w * h,
                                                      H=B * 72, num=B * 4).items()}
    ctx.h2d(d1, g1)
    ctx.h2d(d2, g2)

    def step():
        ctx.flow_warp_diff_batch_dev(B, d1, d2, w, h, w, w * h, mdx.FMT_GRAY8, d_next_pts=dout["np"],
                                     d_status=dout["st"], d_vectors=dout["vec"], d_mask=dout["mask"],
                                     d_H=dout["H"], d_num_vectors=dout["num"])

    def timed(k):
        """k steps between barriers + device syncs (the device sync also reports an LK hand-off
        timeout as an error); returns this rank's wall seconds."""
        D.barrier()
        ctx.device_sync()
        t = time.perf_counter()
        for _ in range(k):
            step()
        ctx.device_sync()
        D.barrier()
        return time.perf_counter() - t

    full_steps = 1 if args.only_roofline else args.steps
    for _ in range(0 if args.only_roofline else args.warmup):
        step()
    ctx.device_sync()

    ctx.enable_timing(True)
    el = timed(full_steps)
    px_rate, el_max = throughput(D, float(full_steps * B * w * h), el)
    value = px_rate / 1e6
    px_all = px_rate * el_max
    st = ctx.stage_ms()
    calls = max(st["calls"], 1)
    stages = {k: round(v / calls, 4) for k, v in st.items() if k != "calls"}
    # the last timed step's outputs, checked against the oracle after every timed leg (untimed)
    outs = {k: np.empty(shape, dt) for k, shape, dt in (("np", (B, n, 2), np.float32), ("st", (B, n), np.uint8),
                                                         ("vec", (B, n, 4), np.float64),
                                                         ("mask", (B, h, w), np.uint8), ("H", (B, 9), np.float64),
                                                         ("num", (B,), np.int32))}
    for k, arr in outs.items():
        ctx.d2h(arr, dout[k])
    num = outs["num"]
    fallbacks = ctx.lk_fallbacks()
    # the same steps with call pipelining off (the line's value_unpipelined)
    value_unpiped = None
    if pipe and not args.only_roofline:
        ctx.set_params(call_pipelining=0)
        step()
        el_u = timed(full_steps)
        value_unpiped = round(throughput(D, float(full_steps * B * w * h), el_u)[0] / 1e6, 2)
        ctx.set_params(call_pipelining=1)
    for p in [d1, d2] + list(dout.values()):
        ctx.dev_free(p)
    del g1, g2

    # ---- the whole path at 4K (config C2; the metric names 1080p & 4K): 8 pairs per step
    full4k = None
    if not args.no_4k and not args.only_roofline and args.config == "1080p":
        kw, kh = CONFIGS["4k"]
        KB = 8
        k1, k2, _, _ = make_batch(kw, kh, KB, min(4, KB), SEED0 + 500 + 1000 * D.rank, threads)
        kctx = open_ctx(D, kw, kh, KB, pixel_step=ps, min_vector_size=1.0, call_pipelining=pipe)
        kn = mdx.grid_count(kw, kh, ps)
        f1, f2 = kctx.dev_alloc(k1.nbytes), kctx.dev_alloc(k2.nbytes)
        # every output, as the headline step writes them
        fo = {k: kctx.dev_alloc(sz) for k, sz in dict(np=KB * kn * 8, st=KB * kn, vec=KB * kn * 32,
                                                      mask=KB * kw * kh, H=KB * 72, num=KB * 4).items()}
        kctx.h2d(f1, k1); kctx.h2d(f2, k2)

        def step4k():
            kctx.flow_warp_diff_batch_dev(KB, f1, f2, kw, kh, kw, kw * kh, mdx.FMT_GRAY8, d_next_pts=fo["np"],
                                          d_status=fo["st"], d_vectors=fo["vec"], d_mask=fo["mask"], d_H=fo["H"],
                                          d_num_vectors=fo["num"])

        for _ in range(max(1, args.warmup)):
            step4k()
        kctx.device_sync()
        D.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step4k()
        kctx.device_sync()
        D.barrier()
        rate4k, el4k = throughput(D, float(args.steps * KB * kw * kh), time.perf_counter() - t0)
        full4k = dict(workload=f"{kw}x{kh} gray pairs, whole reference path (max_level 5 -> 5 levels)", batch_per_gpu=KB,
                      value=round(rate4k / 1e6, 2), unit="Mpixels/s", ms_per_step=round(el4k / args.steps * 1e3, 3),
                      outputs="next_pts, status, Vec4d, mask, H, num_vectors (as the headline step)",
                      lk_fallbacks=kctx.lk_fallbacks())
        for p in [f1, f2] + list(fo.values()):
            kctx.dev_free(p)
        kctx.close()
        del k1, k2

    # ---- MDX_FIT_RANSAC (not in the reference; parity with it N/A): the headline step with the
    # deterministic RANSAC fit instead of first-4, so the warp runs on a real, projective fit
    ransac = None
    if not args.no_ransac and not args.only_roofline and args.config == "1080p":
        rkw = dict(pixel_step=ps, min_vector_size=1.0, call_pipelining=pipe, fit_mode=mdx.FIT_RANSAC)
        qg1, qg2, _, quniq = make_batch(w, h, B, unique, SEED0 + 1000 * D.rank, threads)
        qctx = open_ctx(D, w, h, B, **rkw)
        q1, q2 = qctx.dev_alloc(qg1.nbytes), qctx.dev_alloc(qg2.nbytes)
        qo = {k: qctx.dev_alloc(sz) for k, sz in dict(np=B * n * 8, st=B * n, vec=B * n * 32, mask=B * w * h,
                                                      H=B * 72, num=B * 4).items()}
        qctx.h2d(q1, qg1); qctx.h2d(q2, qg2)

        def stepq():
            qctx.flow_warp_diff_batch_dev(B, q1, q2, w, h, w, w * h, mdx.FMT_GRAY8, d_next_pts=qo["np"],
                                          d_status=qo["st"], d_vectors=qo["vec"], d_mask=qo["mask"], d_H=qo["H"],
                                          d_num_vectors=qo["num"])
        for _ in range(max(1, args.warmup)):
            stepq()
        qctx.device_sync()
        qctx.enable_timing(True)
        D.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            stepq()
        qctx.device_sync()
        D.barrier()
        rateq, elq = throughput(D, float(args.steps * B * w * h), time.perf_counter() - t0)
        qs = qctx.stage_ms()
        qst = {k: round(v / max(qs["calls"], 1), 4) for k, v in qs.items() if k in ("classify_fit", "warp_diff")}
        qH = np.empty((B, 9))
        qctx.d2h(qH, qo["H"])
        qpar = None
        if not args.no_parity:
            from oracle import pyoracle   # untimed checker (test infrastructure)
            qpar = {"checked_pairs": 0, "mismatched_pairs": 0}
            qm = np.empty((B, h, w), np.uint8)
            qctx.d2h(qm, qo["mask"])
            for i, (a, b_, _) in enumerate(quniq):
                r = pyoracle.calculate_optical_flow(a, b_, nthreads=host_cores()["available"], pixel_step=ps,
                                                    min_vector_size=1.0, fit_mode=2, simd=True)
                ok = (np.array_equal(qH[i].view(np.uint64), r["H"].ravel().view(np.uint64)) and
                      np.array_equal(qm[i], r["mask"]))
                qpar["checked_pairs"] += 1
                qpar["mismatched_pairs"] += 0 if ok else 1
        ransac = dict(workload=f"{w}x{h} gray x {B}, the headline step with fit_mode MDX_FIT_RANSAC "
                               f"({mdx.default_params().ransac_iters} hypotheses, 3 px): NOT in the reference, "
                               f"parity with the reference N/A (oracle-pinned, bit-exact)",
                      value=round(rateq / 1e6, 2), unit="Mpixels/s", ms_per_step=round(elq / args.steps * 1e3, 3),
                      stage_ms_per_step=qst, H_pair0=qH[0].tolist(),
                      warp_projective=bool(qH[0][6] != 0.0 or qH[0][7] != 0.0), parity_vs_oracle=qpar)
        for p in [q1, q2] + list(qo.values()):
            qctx.dev_free(p)
        qctx.close()
        del qg1, qg2

    # ---- north-star kernel: fused warp+diff at 4K with the generator's true H
    roof = None
    if not args.no_roofline:
        rw, rh = CONFIGS[args.roofline_config]
        RB = args.roofline_batch
        r1, r2, Hr, _ = make_batch(rw, rh, RB, min(4, RB), SEED0 + 77 + 1000 * D.rank, threads)
        Hb = np.ascontiguousarray(np.broadcast_to(Hr, (RB, 3, 3)), dtype=np.float64)
        rctx = open_ctx(D, 64, 64, 1)   # warp-only: no pyramid workspace needed
        e1, e2 = rctx.dev_alloc(r1.nbytes), rctx.dev_alloc(r2.nbytes)
        eH, eM = rctx.dev_alloc(Hb.nbytes), rctx.dev_alloc(RB * rw * rh)
        rctx.h2d(e1, r1); rctx.h2d(e2, r2); rctx.h2d(eH, Hb)
        launch_ms = None
        # warmup: a burst of launches after idle runs in a clock / power transient (k_warp_diff 157 ->
        # 180-190 -> 141 us over its first ~120 launches on the same inputs, the copy probe flat at
        # 121 us: profiles/r05_warp_transient.txt), so each leg is timed after roofline_warmup launches
        rwarm = max(2, args.warmup, args.roofline_warmup)
        cold_ms = None
        if args.roofline_h != "projective":
            # the cold burst, reported beside the warmed figure: the first --steps launches after
            # --cold-idle seconds of idle (the warmup's first launches)
            rctx.device_sync()
            time.sleep(max(0.0, args.cold_idle))
            rctx.enable_timing(True)
            for _ in range(args.steps):
                rctx.warp_diff_dev(RB, e1, e2, rw, rh, rw, rw * rh, eH, eM)
            rctx.device_sync()
            cs0 = rctx.stage_ms()
            cold_ms = cs0["warp_diff"] / max(cs0["calls"], 1)
            rctx.enable_timing(False)
            for _ in range(rwarm):
                rctx.warp_diff_dev(RB, e1, e2, rw, rh, rw, rw * rh, eH, eM)
            rctx.device_sync()
            rctx.enable_timing(True)
            for _ in range(args.steps):
                rctx.warp_diff_dev(RB, e1, e2, rw, rh, rw, rw * rh, eH, eM)
            rctx.device_sync()
            rs = rctx.stage_ms()
            launch_ms = rs["warp_diff"] / max(rs["calls"], 1)
        alg_bytes = 3.0 * RB * rw * rh     # read gray1 + read gray2 + write mask, 1 B/px each
        achieved = alg_bytes / (launch_ms * 1e-3) / 1e9 if launch_ms else None
        # the memory ceiling of this access mix: the same 3 B/px as one linear non-temporal pass
        # (mdx_probe_stream3_dev, same buffers, same event bracketing)
        for _ in range(rwarm):
            rctx.probe_stream3_dev(RB * rw * rh, e1, e2, eM)
        rctx.device_sync()
        rctx.enable_timing(True)
        for _ in range(args.steps):
            rctx.probe_stream3_dev(RB * rw * rh, e1, e2, eM)
        rctx.device_sync()
        cs = rctx.stage_ms()
        copy_ms = cs["warp_diff"] / max(cs["calls"], 1)
        copy_gbs = alg_bytes / (copy_ms * 1e-3) / 1e9
        kt = stamped_pmc(os.path.join(ROOT, "profiles", "warp_kernel_trace.json"), "config", f"{rw}x{rh}x{RB}")
        # the same launch with a projective H (every non-degenerate first-4 fit is projective): the
        # tests' perspective matrix (tests/test_warp_gpu.py "projective"), per-pixel W and 32 / W
        Hp = np.array([[1.002, 0.013, -2.5], [-0.011, 0.995, 1.75], [2.1e-5, -1.3e-5, 1.0]])
        projective = None
        if args.roofline_h != "affine":
            rctx.h2d(eH, np.ascontiguousarray(np.broadcast_to(Hp, (RB, 3, 3)), dtype=np.float64))
            for _ in range(rwarm):
                rctx.warp_diff_dev(RB, e1, e2, rw, rh, rw, rw * rh, eH, eM)
            rctx.device_sync()
            rctx.enable_timing(True)
            for _ in range(args.steps):
                rctx.warp_diff_dev(RB, e1, e2, rw, rh, rw, rw * rh, eH, eM)
            rctx.device_sync()
            ps_ = rctx.stage_ms()
            proj_ms = ps_["warp_diff"] / max(ps_["calls"], 1)
            proj_gbs = alg_bytes / (proj_ms * 1e-3) / 1e9
            pkt = stamped_pmc(os.path.join(ROOT, "profiles", "warp_kernel_trace_projective.json"), "config",
                              f"{rw}x{rh}x{RB}")
            projective = dict(avg_launch_us=round(proj_ms * 1e3, 2), achieved=round(proj_gbs, 1),
                              frac=round(proj_gbs / HBM_PEAK_GBS, 4),
                              launch_over_affine=round(proj_ms / launch_ms, 3) if launch_ms else None,
                              H=Hp.ravel().tolist(),
                              workload=f"{rw}x{rh} gray, {RB} pairs per launch, projective H (M6, M7 != 0)",
                              kernel_trace=({k: pkt[k] for k in ("launch", "k_warp_diff", "k_warp_prep", "source")
                                             if k in pkt} if pkt else None))
            if pkt and kt:
                projective["kernel_trace_launch_over_affine"] = round(
                    pkt["launch"]["avg_us"] / kt["launch"]["avg_us"], 3) if "avg_us" in pkt.get("launch", {}) else None
        pmc = stamped_pmc(args.pmc_json, "config", f"{rw}x{rh}x{RB}")
        traffic = pmc.get("hbm_bytes_per_launch") if pmc else None
        roof = dict(bound="hbm", achieved=round(achieved, 1) if achieved else None, peak=HBM_PEAK_GBS, unit="GB/s",
                    frac=round(achieved / HBM_PEAK_GBS, 4) if achieved else None, traffic=traffic, kernel="k_warp_diff",
                    workload=f"{rw}x{rh} gray, {RB} pairs per launch, true H (affine), 3 B/px algorithmic",
                    avg_launch_us=round(launch_ms * 1e3, 2) if launch_ms else None,
                    timed_launches=args.steps, warmup_launches=rwarm,
                    cold_burst=(dict(avg_launch_us=round(cold_ms * 1e3, 2),
                                     frac=round(alg_bytes / (cold_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                     what=f"the first {args.steps} launches after {args.cold_idle:g} s idle, before "
                                          f"the warmup (clock / power transient: profiles/r06_warp_burst.txt)")
                                if cold_ms else None),
                    algorithmic_bytes_per_launch=int(alg_bytes),
                    copy_ceiling=dict(achieved=round(copy_gbs, 1), avg_launch_us=round(copy_ms * 1e3, 2),
                                      what="linear 3 B/px pass, 16 B/lane, non-temporal (k_stream3)"),
                    copy_ceiling_frac=round(copy_gbs / HBM_PEAK_GBS, 4),
                    frac_of_copy_ceiling=round(achieved / copy_gbs, 4) if achieved else None,
                    kernel_trace=({k: kt[k] for k in ("launch", "k_warp_diff", "k_warp_prep", "k_stream3",
                                                       "frac_of_copy_ceiling", "source") if k in kt}
                                  if kt else None),
                    projective=projective)
        for p in (e1, e2, eH, eM):
            rctx.dev_free(p)
        rctx.close()
        del r1, r2

    parity = None
    if not args.only_roofline and not args.no_parity:
        parity = check_outputs(uniq, outs, B, w, h, ps, host_cores()["available"])
    cpu = cpu1 = cpu_scalar = None
    if D.world == 1 and not args.no_cpu:
        hc = host_cores()
        cpu = cpu_baseline(uniq, w, h, args.cpu_seconds, hc["available"])   # every CPU this job may use, SSE2
        cpu.update(nproc=hc["nproc"], cgroup_cpu_quota=hc["cgroup_cpu_quota"])
        cpu1 = cpu_baseline(uniq, w, h, args.cpu_seconds / 2, 1)          # one core, SSE2
        cpu_scalar = cpu_baseline(uniq, w, h, args.cpu_seconds / 2, hc["available"], simd=False)
    live = None
    if D.world == 1 and not args.no_live and not args.only_roofline:
        live = live_leg(D.local_rank, w, h, threads, with_cpu=not args.no_cpu)

    lk_share = stages["lk"] / stages["total"] if stages["total"] > 0 else None
    # VALU roofline of the dominant stage (LK): algorithmic wave-instructions of the
    # step's B pairs over the LK stage's HIP-event time, against the chip's VALU issue rate
    lk_roof = None
    if not args.only_roofline and not args.no_lk_roofline and stages.get("lk", 0) > 0:
        wk = lk_work(ctx.device, w, h, ps, uniq)
        alg_wave = wk["valu_lane_instr_per_pair"] * B / 64.0
        ach = alg_wave / (stages["lk"] * 1e-3)
        lk_roof = dict(bound="valu", unit="wave-instr/s", achieved=round(ach, 1), peak=VALU_PEAK_WAVE_INSTR,
                       frac=round(ach / VALU_PEAK_WAVE_INSTR, 4),
                       peak_basis="4 cycles per wave64 VALU instruction (one wave's issue cost, measured op mix)",
                       peak_2cyc=VALU_PEAK_WAVE_INSTR_2CYC, frac_2cyc=round(ach / VALU_PEAK_WAVE_INSTR_2CYC, 4),
                       peak_2cyc_basis="2 cycles per wave64 VALU instruction (SIMD rate, MI355X_MICROARCH.md:54)",
                       stage_ms=stages["lk"],
                       algorithmic_wave_instr_per_step=round(alg_wave, 1), per_element=dict(
                           iteration=LK_VALU_PER_ELEM_ITER, gradient_sums=LK_VALU_PER_ELEM_A),
                       workload=f"{B} pairs {w}x{h}, pixel_step {ps}, {wk['levels']} levels", **{
                           k: v for k, v in wk.items() if k not in ("valu_lane_instr_per_pair", "levels")})
        pj = stamped_pmc(os.path.join(ROOT, "profiles", "pmc_lk_iter.json"), "config", f"{w}x{h}x{B}_ps{ps}")
        lk_roof["executed_wave_instr_per_step"] = pj.get("sq_insts_valu_per_step") if pj else None
        lk_roof["executed_over_algorithmic"] = round(pj["sq_insts_valu_per_step"] / alg_wave, 3) if pj else None
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "Mpixels/s",
        "n_gpus": devs["n_gpus"],
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el_max / full_steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (mdx_synth_pair: textured scene, affine camera motion + moving patch + noise)",
        "config": {"workload": f"{w}x{h} gray frame pairs through the full reference path (pyramid + Scharr, "
                               f"pyramidal LK 40x40 / 10 iters, first-4 perspective fit, warp+absdiff+threshold)",
                   "frame": f"{w}x{h}", "pixel_step": ps, "grid_points_per_pair": mdx.grid_count(w, h, ps),
                   "batch_per_gpu": B, "unique_pairs_per_gpu": unique, "call_pipelining": bool(pipe),
                   "parallelism": f"{D.world} independent stream shard(s), one per GPU, no collectives"},
        "value_unpipelined": value_unpiped,
        "parity_checked_pairs": parity["checked_pairs"] if parity else 0,
        "parity": parity,
        "roofline": roof,
        "cpu_baseline": cpu,
        "cpu_baseline_1core": cpu1,
        "cpu_baseline_scalar": cpu_scalar,
        "ranks": devs["ranks"],
        "devices": devs["devices"],
        "build": mdx._lib.build_info(),
        "stage_ms_per_step": stages,
        "dominant_kernel": {"name": "k_lk_class + k_lk_A + k_lk_iter (LK stage)",
                            "share_of_step": round(lk_share, 4) if lk_share else None,
                            "bound": "valu/lds (exact-order float chains), not hbm",
                            "points_per_s": round(px_all / (w * h) * mdx.grid_count(w, h, ps) / el_max, 1),
                            "roofline": lk_roof},
        "num_vectors_pair0": int(num[0]),
        "lk_fallbacks": fallbacks,
        "full_path_4k": full4k,
        "full_path_ransac": ransac,
        "live_path": live,
    }
    if D.rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    D.close()


if __name__ == "__main__":
    main()
