"""Tuning study (not product): time the warped integrate kernel variants (OFX_INT_VARIANT) at 512^3."""
import os, sys, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from occlusionfusion_amd import synthetic as S
from occlusionfusion_amd.pipeline import FusionPipeline
dev = torch.device("cuda", 0)
seq = S.SyntheticSequence.build(2000, seed=3)
pipe = FusionPipeline(seq, (-1.024, -1.024, 0.5), 0.004, (512, 512, 512), device=dev)
f0 = pipe.prepare(0); f1 = pipe.prepare(1)
pipe.integrate_source(f0)
pipe.solve(f1)
pipe.integrate(f1, 1)
torch.cuda.synchronize()
res = {}
t = 2
for var in sys.argv[1:] or ["0", "1", "2", "0"]:
    os.environ["OFX_INT_BPW"] = var
    pipe.vol.kernel_timer = []
    for _ in range(40):
        pipe.integrate(f1, t)
        t += 1
    torch.cuda.synchronize()
    ts = [a.elapsed_time(b) * 1e3 for a, b in pipe.vol.kernel_timer[5:]]
    res[var] = (float(np.median(ts)), float(np.min(ts)))
    print(var, res[var], flush=True)
