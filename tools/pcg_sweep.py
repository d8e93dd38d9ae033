"""Tuning sweep (not part of the product): PCG tolerance accuracy and per-iteration latency."""
import os, sys, json, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from occlusionfusion_amd import synthetic as S
from occlusionfusion_amd.pipeline import FusionPipeline
from occlusionfusion_amd import GaussNewtonSolver
dev = torch.device("cuda", 0)
seq = S.SyntheticSequence.build(2000, seed=3)
pipe = FusionPipeline(seq, (-1.024, -1.024, 0.5), 0.004, (64, 64, 64), device=dev)
f = pipe.prepare(3)
args = (pipe.nodes_t, pipe.edges_t, pipe.ew_t, f.tpos, f.conf, f.src, f.anchors, f.weights, f.tgt, pipe.intr)
ref = GaussNewtonSolver(len(seq.nodes), 10000, pcg_tol=1e-11).optimize(*args)
out = {}
for tol in [1e-5, 1e-6, 1e-7, 1e-8]:
    s = GaussNewtonSolver(len(seq.nodes), 10000, pcg_tol=tol)
    r = s.optimize(*args)
    s.timing(True); r = s.optimize(*args); ms, n, _ = s.timing(False)
    out[tol] = dict(dt=(r["node_translations"] - ref["node_translations"]).abs().max().item(),
                    dr=(r["node_rotations"] - ref["node_rotations"]).abs().max().item(),
                    iters=r["convergence_info"]["pcg_iterations"], us_per_launch=1e3 * ms / n, launches=n)
print(json.dumps({str(k): v for k, v in out.items()}))
