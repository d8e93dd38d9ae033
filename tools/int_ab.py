"""Tuning study (not product): warped integrate kernel time under an environment switch read per launch, the settings
interleaved launch by launch in one process on the bench scene (config 3 by default). Default switch OFX_INT_GENERIC
(the generic k_integrate<1,1,0> against the specialised k_integrate_pal4, plus the source-frame pass); any switch the
integrate reads per launch (round 4: OFX_INT_TAB, separable warp tables, 113.9 vs 90.2 us: dropped).

    python tools/int_ab.py [--config 3] [--var OFX_INT_GENERIC --vals 1 0] [--reps 40]
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
ap.add_argument("--var", default="OFX_INT_GENERIC")
ap.add_argument("--vals", nargs="+", default=["1", "0"])
ap.add_argument("--reps", type=int, default=30)
a = ap.parse_args()
c = S.BASELINE_CONFIGS[a.config]
dev = torch.device("cuda", 0)
seq = S.config_sequence(a.config, device=dev)
D = c["dims"]
pipe = FusionPipeline(seq, c["origin"], c["voxel"], (D, D, D), device=dev)
pipe.integrate_source(pipe.prepare(0))
f1 = pipe.prepare(1)
pipe.solve(f1)
torch.cuda.synchronize()


def setv(v):
    if v == "":
        os.environ.pop(a.var, None)
    else:
        os.environ[a.var] = v


res = {v: [] for v in a.vals}
t = 1
for rep in range(a.reps):
    for v in a.vals:
        setv(v)
        pipe.vol.integrate_timing(True)
        pipe.integrate(f1, t)
        t += 1
        torch.cuda.synchronize()
        ms, n = pipe.vol.integrate_timing(False)
        res[v].append(ms * 1e3 / n)
if a.var == "OFX_INT_GENERIC":   # source frame (dense pass) on a scratch volume of the same grid, both kernels
    from occlusionfusion_amd import TSDFVolume  # noqa: E402
    scratch = TSDFVolume.from_grid(c["origin"], c["voxel"], (D, D, D), pipe.intr, pipe.fopt, device=dev)
    f0 = pipe.prepare(0)
    for v in a.vals:
        res["src " + v] = []
    for rep in range(12):
        for v in a.vals:
            setv(v)
            if hasattr(scratch, "frame_id"):
                del scratch.frame_id
            scratch.update(f0.im, 0)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            scratch.integrate_device()
            e1.record()
            torch.cuda.synchronize()
            res["src " + v].append(e0.elapsed_time(e1) * 1e3)
os.environ.pop(a.var, None)
for k, v in res.items():
    v = np.array(v[3:])
    print(f"{a.var}={k}: median {np.median(v):.1f} us  min {v.min():.1f} us", flush=True)
