"""Tuning (not product): in-process A/B of environment switches read per solve (e.g. OFX_GN_PIPE), alternating frame by
frame on the bench's config-3 sequence, so that run-level spread (whole processes land at ~5.0 or ~5.3 us per PCG
launch) cancels. Prints mean ms per frame (solve + integrate, stream events) per setting.

    python tools/ab_inproc.py OFX_GN_PIPE 0 1 [--frames 120]
    python tools/ab_inproc.py prefetch_lead 0 1 2 --block 8   # a solver attribute, switched every 8 frames
    python tools/ab_inproc.py param:pcg_tol 1e-6 3e-6 --sweep 3   # a GN parameter

--block B: switch every B frames and leave the first frame of each block out (a setting that acts across the
frame boundary, such as when the next frame's prefetched setup starts, then counts only against itself).
--sweep R: instead, run the same frames once per setting, R rounds (settings in turn); also reports the mean per-frame
difference to the first setting over identical frames.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("var")
    ap.add_argument("values", nargs="+")
    ap.add_argument("--frames", type=int, default=120)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--block", type=int, default=1)
    ap.add_argument("--sweep", type=int, default=0)
    a = ap.parse_args()
    from occlusionfusion_amd import synthetic as S
    from occlusionfusion_amd.pipeline import FusionPipeline
    dev = torch.device("cuda", 0)
    cfg = S.BASELINE_CONFIGS[a.config]
    seq = S.config_sequence(a.config, device=dev)
    D = cfg["dims"]
    pipe = FusionPipeline(seq, cfg["origin"], cfg["voxel"], (D, D, D), device=dev)
    total = a.frames + 4
    frames = [pipe.prepare(t) for t in range(total + 1)]
    torch.cuda.synchronize()
    pipe.integrate_source(frames[0])
    times = {v: [] for v in a.values}
    marks = []

    def setv(v):
        if a.var == "prefetch_lead":
            pipe.solver.prefetch_lead = int(v)
        elif a.var.startswith("param:"):   # a GN parameter (e.g. param:pcg_tol); use --sweep (prefetches match params)
            pipe.solver.params[a.var[6:]] = float(v)
        else:
            os.environ[a.var] = v

    if a.sweep:
        per = {v: [] for v in a.values}
        launches = {v: [] for v in a.values}   # k_pcg_iter launches and PCG iterations per frame (whole run)
        iters = {v: [] for v in a.values}
        tg = 0   # the volume's frame counter keeps increasing over the repeated frames
        for r in range(a.sweep):
            for v in a.values:
                setv(v)
                pipe.prev_rot = pipe.prev_trans = None   # the same solves each run: frame 1 from the rest pose
                ev, outs = [], []
                pipe.solver.timing(True)
                for t in range(1, total):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    outs.append(pipe.solve(frames[t], frames[t + 1]))
                    tg += 1
                    pipe.integrate(frames[t], tg)
                    e1.record()
                    ev.append((e0, e1))
                pipe.solver.drain()
                torch.cuda.synchronize()
                per[v].append(np.array([e0.elapsed_time(e1) for e0, e1 in ev[4:]]))
                _, nl, _ = pipe.solver.timing(False)
                launches[v].append(nl / len(outs))
                iters[v].append(float(np.mean([int(o["_status"][2].item()) for o in outs])))
        base = np.stack(per[a.values[0]])
        out = {}
        for v in a.values:
            x = np.stack(per[v])
            out[v] = {"ms_per_frame": float(x.mean()), "run_means": [float(q) for q in x.mean(1)],
                      "paired_diff_ms": float((x - base).mean()), "n": int(x.size),
                      "launches_per_frame": float(np.mean(launches[v])), "iters_per_frame": float(np.mean(iters[v]))}
        print(json.dumps({"var": a.var, "sweep": a.sweep, "results": out}))
        return
    for t in range(1, total):
        v = a.values[(t // a.block) % len(a.values)]
        setv(v)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        pipe.solve(frames[t], frames[t + 1])
        pipe.integrate(frames[t], t)
        e1.record()
        if t > 4 and (a.block == 1 or t % a.block != 0):
            marks.append((v, e0, e1))
    pipe.solver.drain()
    torch.cuda.synchronize()
    for v, e0, e1 in marks:
        times[v].append(e0.elapsed_time(e1))
    out = {v: {"ms_per_frame": float(np.mean(x)), "median": float(np.median(x)), "n": len(x)} for v, x in times.items()}
    print(json.dumps({"var": a.var, "results": out}))


if __name__ == "__main__":
    main()
