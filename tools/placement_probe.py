"""Tuning probe (not product): is the run-to-run PCG launch bimodality (whole processes at ~4.6 or ~5.2 us per
launch) a property of the process or of where the solver's buffers landed? Builds K frame loops one after
another in ONE process (each with its own solver handles, buffers and volume; the earlier ones stay allocated so
every loop gets fresh memory) and reports each loop's mean PCG launch time over the same frames.

    python tools/placement_probe.py [--loops 6] [--frames 40] [--config 3]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--loops", type=int, default=6)
    ap.add_argument("--frames", type=int, default=40)
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--free", action="store_true", help="drop each loop before building the next")
    a = ap.parse_args()
    from occlusionfusion_amd import synthetic as S
    from occlusionfusion_amd.pipeline import FusionPipeline
    dev = torch.device("cuda", 0)
    cfg = S.BASELINE_CONFIGS[a.config]
    seq = S.config_sequence(a.config, device=dev)
    D = cfg["dims"]
    keep, out = [], []
    for k in range(a.loops):
        pipe = FusionPipeline(seq, cfg["origin"], cfg["voxel"], (D, D, D), device=dev)
        frames = [pipe.prepare(t) for t in range(a.frames + 2)]
        pipe.integrate_source(frames[0])
        for t in range(1, 4):   # warm-up
            pipe.step(frames[t], t, next_fi=frames[t + 1])
        pipe.solver.drain()
        torch.cuda.synchronize()
        pipe.solver.timing(True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for t in range(4, a.frames + 1):
            pipe.step(frames[t], t, next_fi=frames[t + 1])
        e1.record()
        pipe.solver.drain()
        torch.cuda.synchronize()
        ms, launches, iters = pipe.solver.timing(False)
        n = a.frames - 3
        out.append({"loop": k, "us_per_launch": 1e3 * ms / max(launches, 1), "launches_per_frame": launches / n,
                    "ms_per_frame": e0.elapsed_time(e1) / n})
        print(json.dumps(out[-1]), flush=True)
        if a.free:
            del pipe, frames
            torch.cuda.empty_cache()
        else:
            keep.append((pipe, frames))
    print(json.dumps({"loops": out}))


if __name__ == "__main__":
    main()
