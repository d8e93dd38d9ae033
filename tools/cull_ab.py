"""Tuning (not product): the warped integrate with and without the per-frame brick cull (TSDFVolume.brick_cull), the
settings alternated launch by launch on one frame of the bench scene (config 3 by default, frame 1 after its solve);
timed by the library's integrate events (with the cull: its three kernels). The volume is restored before each launch.

    python tools/cull_ab.py [--config 3] [--reps 30]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from occlusionfusion_amd import synthetic as S  # noqa: E402
from occlusionfusion_amd.pipeline import FusionPipeline  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=3)
ap.add_argument("--reps", type=int, default=30)
ap.add_argument("--frame", type=int, default=1)
a = ap.parse_args()
c = S.BASELINE_CONFIGS[a.config]
dev = torch.device("cuda", 0)
seq = S.config_sequence(a.config, device=dev)
D = c["dims"]
pipe = FusionPipeline(seq, c["origin"], c["voxel"], (D, D, D), device=dev)
pipe.integrate_source(pipe.prepare(0))
fr = pipe.prepare(a.frame)
pipe.solve(fr)
pipe.wf.set_node_transforms(pipe.prev_rot, pipe.prev_trans)
pipe.wf.frame_id = a.frame
vol = pipe.vol
vol.update(fr.im, a.frame)
torch.cuda.synchronize()
keep = tuple(x.clone() for x in (vol.tsdf_b, vol.weight_b, vol.color_b))
res = {True: [], False: []}
for r in range(a.reps):
    for cull in (True, False):
        vol.tsdf_b.copy_(keep[0]); vol.weight_b.copy_(keep[1]); vol.color_b.copy_(keep[2])
        vol.brick_cull = cull
        torch.cuda.synchronize()
        vol.integrate_timing(True)
        vol.integrate_device(count_updates=True)
        torch.cuda.synchronize()
        ms, n = vol.integrate_timing(False)
        res[cull].append(1e3 * ms / max(1, n))
n_list = pipe.wf.skin_tsdf_cache().n_list
kept = int(vol._cull[1][:n_list].sum().item())
print({"config": a.config, "listed": n_list, "kept": kept,
       "us_cull": float(np.median(res[True])), "us_nocull": float(np.median(res[False]))}, flush=True)
