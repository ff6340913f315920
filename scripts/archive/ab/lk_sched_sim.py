"""Offline model of the LK iteration kernel's scheduling waste, from measured per-point iteration
counts (gpurun_out/lk_iters.npz, written on the GPU box by scripts/lk_iters.py).

A slot runs one work unit at a time; every iteration step costs the whole slot (its quads execute
in lockstep).  Schemes:
  group G        G consecutive class members of one grid row, the slot steps max(iters) times
                 (the kernel's scheme: G = 8 at level 0, 4 above);
  slide G,S,K    runs cut into K-member segments; G quads walk a segment, a finished quad takes
                 the next member while it lies within S members of the leftmost active one (the
                 union then spans S members).
Prints executed/ideal iteration ratios and, for a persistent queue of 6144 waves, the per-level
makespan in steps (equal-speed slots: pessimistic for tails, where fewer waves run faster).
Usage: python scripts/lk_sched_sim.py
"""
import heapq

import numpy as np

W, H, PS, NLEV, PAIRS = 1920, 1080, 10, 5, 32
NX, NY = (W + PS - 1) // PS, (H + PS - 1) // PS


def runs_of(buf, L):
    it = buf[L, :, 2].reshape(NX, NY).astype(int)
    m = (1 << L) - 1
    runs = []
    for gy in range(NY):
        cls = {}
        for gx in range(NX):
            cls.setdefault((gx * PS) & m, []).append(it[gx, gy])
        runs += list(cls.values())
    return runs


def slide_steps(r, G, S):
    n, rem, nxt, quads, steps = len(r), list(r), 0, [None] * G, 0

    def fill():
        nonlocal nxt
        for qi in range(G):
            if quads[qi] is None:
                while nxt < n and rem[nxt] == 0:
                    nxt += 1
                if nxt >= n:
                    return
                act = [x for x in quads if x is not None]
                if nxt - (min(act) if act else nxt) < S:
                    quads[qi] = nxt
                    nxt += 1
    fill()
    while any(x is not None for x in quads):
        steps += 1
        for qi in range(G):
            if quads[qi] is not None:
                rem[quads[qi]] -= 1
                if rem[quads[qi]] == 0:
                    quads[qi] = None
        fill()
    return steps


def makespan(units, nslots):
    h = [0] * nslots
    for s in units:
        heapq.heappush(h, heapq.heappop(h) + s)
    return max(h)


def main():
    d = np.load("gpurun_out/lk_iters.npz")
    bufs = [d["1920x1080_ps10_s1"], d["1920x1080_ps10_s2"]]
    for scheme in ["group", "slide K=8", "slide K=16", "slide K=32", "slide unsegmented"]:
        work = ideal = span = 0
        for L in range(NLEV):
            G = 8 if L == 0 else 4
            S = 8 if L == 0 else 5
            units = []
            for p in range(PAIRS):
                runs = runs_of(bufs[p % 2], L)
                ideal += sum(map(sum, runs))
                for r in runs:
                    if scheme == "group":
                        units += [max(r[q:q + G]) for q in range(0, len(r), G)]
                    else:
                        K = len(r) if "unseg" in scheme else int(scheme.split("=")[1])
                        units += [slide_steps(r[q:q + K], G, S) for q in range(0, len(r), K)]
            work += sum(units) * G
            span += makespan(units, 6144 * (64 // (4 * G)))
        print(f"{scheme:18s} executed/ideal {work / ideal:.3f}  sum of level makespans {span}")


if __name__ == "__main__":
    main()
