"""Tuning study (not product): warped integrate kernel time, specialised k_integrate_pal4 vs the generic
k_integrate<1,1,0> (OFX_INT_GENERIC=1), interleaved in one process on the bench scene (config 3 by default)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from occlusionfusion_amd import synthetic as S  # noqa: E402
from occlusionfusion_amd.pipeline import FusionPipeline  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
c = S.BASELINE_CONFIGS[cfg]
dev = torch.device("cuda", 0)
seq = S.config_sequence(cfg)
D = c["dims"]
pipe = FusionPipeline(seq, c["origin"], c["voxel"], (D, D, D), device=dev)
pipe.integrate_source(pipe.prepare(0))
f1 = pipe.prepare(1)
pipe.solve(f1)
torch.cuda.synchronize()
res = {"generic": [], "pal4": []}
t = 1
for rep in range(30):
    for var in ("generic", "pal4"):
        if var == "generic":
            os.environ["OFX_INT_GENERIC"] = "1"
        else:
            os.environ.pop("OFX_INT_GENERIC", None)
        pipe.vol.integrate_timing(True)
        pipe.integrate(f1, t)
        t += 1
        torch.cuda.synchronize()
        ms, n = pipe.vol.integrate_timing(False)
        res[var].append(ms * 1e3 / n)
# source frame (dense pass) on a scratch volume of the same grid, both kernels interleaved
from occlusionfusion_amd import TSDFVolume  # noqa: E402
scratch = TSDFVolume.from_grid(c["origin"], c["voxel"], (D, D, D), pipe.intr, pipe.fopt, device=dev)
f0 = pipe.prepare(0)
res.update({"src_generic": [], "src_table": []})
for rep in range(12):
    for var in ("src_generic", "src_table"):
        if var == "src_generic":
            os.environ["OFX_INT_GENERIC"] = "1"
        else:
            os.environ.pop("OFX_INT_GENERIC", None)
        if hasattr(scratch, "frame_id"):
            del scratch.frame_id
        scratch.update(f0.im, 0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        scratch.integrate_device()
        e1.record()
        torch.cuda.synchronize()
        res[var].append(e0.elapsed_time(e1) * 1e3)
os.environ.pop("OFX_INT_GENERIC", None)
for k, v in res.items():
    v = np.array(v[3:])
    print(f"{k}: median {np.median(v):.1f} us  min {v.min():.1f} us", flush=True)
