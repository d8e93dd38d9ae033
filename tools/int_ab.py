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
        pipe.vol.kernel_timer = []
        pipe.integrate(f1, t)
        t += 1
        torch.cuda.synchronize()
        a, b = pipe.vol.kernel_timer[0]
        res[var].append(a.elapsed_time(b) * 1e3)
for k, v in res.items():
    v = np.array(v[3:])
    print(f"{k}: median {np.median(v):.1f} us  min {v.min():.1f} us", flush=True)
