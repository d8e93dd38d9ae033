"""Chunk-sizing study for the PCG host loop (CPU, not product): replays measured per-GN-step PCG iteration counts
(tools/pcg_counts.py -> gpurun_out/pcg_counts_c3.json) through first-chunk rules and reports, per frame, the drained
launches (enqueued after the converging one: each ends after its first memory trip, ~1.6 us) and the top-ups (a chunk
that ran out before convergence: the host enqueues more; without lookahead the stream idles for the host's reaction).

  python tools/chunk_sim.py gpurun_out/pcg_counts_c3.json
"""
import json
import sys

import numpy as np


def replay(counts, first, topup=8, name=""):
    """first(f, k, hist) -> first chunk of frame f, step k (hist: counts of the frames before f and of this
    frame's steps before k)."""
    drains, tops = [], []
    for f in range(1, len(counts)):
        d = t = 0
        for k, c in enumerate(counts[f]):
            if c <= 0:
                continue
            n = max(1, first(f, k, counts))
            while n < c + 1:          # launch i tests the state after i iterations: c + 1 launches needed
                n += topup
                t += 1
            d += n - (c + 1)
        drains.append(d)
        tops.append(t)
    print(f"{name:44s} drained {np.mean(drains):6.1f} per frame, top-ups {np.mean(tops):5.2f} per frame")


def main():
    counts = json.load(open(sys.argv[1]))["counts"]
    print(f"{len(counts)} frames, {np.mean([sum(c) for c in counts]):.1f} iterations per frame")
    prev = lambda f, k, C: C[f - 1][k]
    replay(counts, lambda f, k, C: prev(f, k, C) + 4, name="rounds 1-3: previous frame's count + 4")
    for m in (0, 2):
        replay(counts, lambda f, k, C, m=m: prev(f, k, C) + m, name=f"previous + {m}")

    # the product rule since round 4 (gn.hip gn_pcg, OFX_PCG_RATIO): step 0 keeps previous + 4, later steps scale the
    # previous frame's count by this frame's step-0 ratio (clamped to [0.5, 2]) + m
    def ratio(f, k, C, m=0, upto=lambda k: 1):
        if k == 0:
            return C[f - 1][0] + 4
        j = upto(k)
        r = min(2.0, max(0.5, sum(C[f][:j]) / max(1, sum(C[f - 1][:j]))))
        return int(round(C[f - 1][k] * r)) + m
    for m in (0, 2, 4):
        replay(counts, lambda f, k, C, m=m: ratio(f, k, C, m), name=f"product: ratio of step 0 + {m}")
        replay(counts, lambda f, k, C, m=m: ratio(f, k, C, m, upto=lambda k: k),
               name=f"ratio of steps 0..k-1 (cumulative) + {m}")

    def minlast(f, k, C, w=3, m=0):
        return min(C[g][k] for g in range(max(0, f - w), f)) + m
    for w in (2, 3, 5):
        for tp in (4, 8):
            replay(counts, lambda f, k, C, w=w: minlast(f, k, C, w), topup=tp,
                   name=f"min of last {w} frames, top-up {tp}")

    def under(f, k, C, frac=0.9):
        return int(C[f - 1][k] * frac)
    for fr in (0.8, 0.9):
        for tp in (2, 4):
            replay(counts, lambda f, k, C, fr=fr: under(f, k, C, fr), topup=tp, name=f"previous x {fr}, top-up {tp}")


if __name__ == "__main__":
    main()
