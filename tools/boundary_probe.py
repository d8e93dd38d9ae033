"""Tuning probe (not product): does the GPU wait for the host at the frame boundary? Per frame of the bench loop
(config 3, prefetch on): event A after the solve's enqueue, B after the integrate's, C at the start of the next
frame's solve call. B -> C on the GPU clock is the time the stream sat idle because the host had not yet enqueued
the next frame (0 when the host is ahead); A -> B is the integrate's stream time. Host-side: Python time of the
integrate call and of the next optimize() up to its return.

    python tools/boundary_probe.py [--frames 60]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=60)
    ap.add_argument("--config", type=int, default=3)
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
    pipe.integrate_source(frames[0])
    torch.cuda.synchronize()
    ev = lambda: torch.cuda.Event(enable_timing=True)
    marks, host = [], []
    prev_b = None
    for t in range(1, total):
        c = ev()
        c.record()
        h0 = time.perf_counter()
        pipe.solve(frames[t], frames[t + 1])
        h1 = time.perf_counter()
        ea = ev()
        ea.record()
        pipe.integrate(frames[t], t)
        h2 = time.perf_counter()
        eb = ev()
        eb.record()
        if t > 4:
            marks.append((prev_b, c, ea, eb))
            host.append((h1 - h0, h2 - h1))
        prev_b = eb
    pipe.solver.drain()
    torch.cuda.synchronize()
    idle = np.array([pb.elapsed_time(c) for pb, c, _, _ in marks]) * 1e3
    integ = np.array([x.elapsed_time(y) for _, _, x, y in marks]) * 1e3
    solve = np.array([c.elapsed_time(x) for _, c, x, _ in marks]) * 1e3
    hs = np.array(host) * 1e6
    print(json.dumps({"frames": len(marks), "stream_idle_before_solve_us": {"mean": float(idle.mean()),
                      "median": float(np.median(idle)), "max": float(idle.max())},
                      "integrate_stream_us": float(integ.mean()), "solve_stream_us": float(solve.mean()),
                      "host_solve_call_us": float(hs[:, 0].mean()), "host_integrate_call_us": float(hs[:, 1].mean())}))


if __name__ == "__main__":
    main()
