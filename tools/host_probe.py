"""Tuning probe (not product): host time of the frame loop's per-frame Python between two solves — the integrate's
enqueue (FusionPipeline.integrate, overlapped) and the solve call's own Python before its first kernel — on the
bench's config-3 workload. With the solves latency-bound and host-driven, this time is a GPU gap between frames.
    python tools/host_probe.py
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from occlusionfusion_amd import synthetic as S  # noqa: E402
from occlusionfusion_amd.pipeline import FusionPipeline  # noqa: E402

dev = torch.device("cuda", 0)
c = S.BASELINE_CONFIGS[3]
seq = S.config_sequence(3, device=dev)
D = c["dims"]
pipe = FusionPipeline(seq, c["origin"], c["voxel"], (D, D, D), device=dev, overlap=True)
frames = [pipe.prepare(t) for t in range(32)]
pipe.integrate_source(frames[0])
torch.cuda.synchronize()
t_int, t_stage, t_solve = [], [], []
for t in range(1, 30):
    a = time.perf_counter()
    pipe.vol.stage(frames[t].im)
    b = time.perf_counter()
    out = pipe.solver.optimize(pipe.nodes_t, pipe.edges_t, pipe.ew_t, frames[t].tpos, frames[t].conf, frames[t].src,
                               frames[t].anchors, frames[t].weights, frames[t].tgt, pipe.intr, prev_rot=pipe.prev_rot,
                               prev_trans=pipe.prev_trans, sync=False, prefetch=pipe.problem(frames[t + 1]))
    pipe.prev_rot, pipe.prev_trans = out["node_rotations"], out["node_translations"]
    c_ = time.perf_counter()
    pipe.integrate(frames[t], t, count_updates=True)
    d = time.perf_counter()
    if t > 5:
        t_stage.append(b - a); t_solve.append(c_ - b); t_int.append(d - c_)
torch.cuda.synchronize()
print(f"host us per frame: stage {1e6 * np.median(t_stage):.1f}, solve call {1e6 * np.median(t_solve):.1f}, "
      f"integrate enqueue {1e6 * np.median(t_int):.1f}")
# the pieces of the overlapped integrate's enqueue
import ctypes  # noqa: E402
tt = {k: [] for k in ("events+wait", "record_stream", "set_transforms", "update", "packed_nodes", "skin_cache", "lib call")}
vol, wf = pipe.vol, pipe.wf
s_ = pipe.int_stream
for t in range(1, 25):
    k = 1 + (t % 28)
    vol.stage(frames[k].im)
    a = time.perf_counter()
    ev = torch.cuda.Event(); ev.record(); s_.wait_event(ev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    b = time.perf_counter()
    st = vol._staged
    for x in (pipe.prev_rot, pipe.prev_trans, st[1], st[2]):
        x.record_stream(s_)
    c_ = time.perf_counter()
    with torch.cuda.stream(s_):
        wf.set_node_transforms(pipe.prev_rot, pipe.prev_trans)
        d = time.perf_counter()
        wf.frame_id = k
        vol.frame_id = k - 1
        vol.update(frames[k].im, k)
        e = time.perf_counter()
        nodes = wf.packed_nodes()
        f = time.perf_counter()
        cache = wf.skin_tsdf_cache()
        g = time.perf_counter()
        vol.integrate_device(count_updates=True)
        h = time.perf_counter()
    for key, v in zip(tt, (b - a, c_ - b, d - c_, e - d, f - e, g - f, h - g)):
        tt[key].append(v)
torch.cuda.synchronize()
print("host us per piece:", {k: round(1e6 * float(np.median(v)), 1) for k, v in tt.items()})
