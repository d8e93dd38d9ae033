"""Tuning probe (not product): host (Python) time of the frame loop's integrate call, by sub-step, on the bench's
config 3 loop (tools/boundary_probe.py showed the GPU waiting for it). Each sub-step is timed with perf_counter
inside the real frame loop (no syncs added).

    python tools/integrate_host_probe.py [--frames 60]
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
    a = ap.parse_args()
    from occlusionfusion_amd import synthetic as S
    from occlusionfusion_amd.pipeline import FusionPipeline
    dev = torch.device("cuda", 0)
    cfg = S.BASELINE_CONFIGS[3]
    seq = S.config_sequence(3, device=dev)
    D = cfg["dims"]
    pipe = FusionPipeline(seq, cfg["origin"], cfg["voxel"], (D, D, D), device=dev)
    total = a.frames + 4
    frames = [pipe.prepare(t) for t in range(total + 1)]
    pipe.integrate_source(frames[0])
    torch.cuda.synchronize()
    vol, wf = pipe.vol, pipe.wf
    keys = ("set_node_transforms", "update", "skin_tsdf_cache", "packed_nodes", "integrate_device_rest", "solve_call")
    acc = {k: [] for k in keys}
    for t in range(1, total):
        q0 = time.perf_counter()
        pipe.solve(frames[t], frames[t + 1])
        q1 = time.perf_counter()
        wf.set_node_transforms(pipe.prev_rot, pipe.prev_trans)
        wf.frame_id = t
        q2 = time.perf_counter()
        vol.update(frames[t].im, t)
        q3 = time.perf_counter()
        wf.skin_tsdf_cache()
        q4 = time.perf_counter()
        wf.packed_nodes()
        q5 = time.perf_counter()
        vol.integrate_device()
        q6 = time.perf_counter()
        if t > 4:
            for k, v in zip(keys, (q2 - q1, q3 - q2, q4 - q3, q5 - q4, q6 - q5, q1 - q0)):
                acc[k].append(v * 1e6)
    pipe.solver.drain()
    torch.cuda.synchronize()
    print(json.dumps({k: float(np.median(v)) for k, v in acc.items()}))


if __name__ == "__main__":
    main()
