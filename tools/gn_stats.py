"""Tuning study (not part of the product): per-GN-step PCG iterations / |b|² / loss along the bench's
frame chain, and the transform deviation of PCG stop-test variants from a tight (1e-11) solve that
starts from the same previous-frame state."""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from occlusionfusion_amd import synthetic as S
from occlusionfusion_amd.pipeline import FusionPipeline
from occlusionfusion_amd import GaussNewtonSolver

dev = torch.device("cuda", 0)
seq = S.SyntheticSequence.build(2000, seed=3)
pipe = FusionPipeline(seq, (-1.024, -1.024, 0.5), 0.004, (64, 64, 64), device=dev)
N = len(seq.nodes)
variants = [("warm1e-7", 1, 1e-7), ("warm3e-7", 1, 3e-7), ("warm1e-6", 1, 1e-6)]
solvers = {}
for name, wm, tol in variants:
    solvers[name] = GaussNewtonSolver(N, 10000, pcg_tol=tol, pcg_warm=bool(wm))
ref = GaussNewtonSolver(N, 10000, pcg_tol=1e-11, pcg_warm=False)
prev_r = prev_t = None
res = []
for t in range(1, 9):
    f = pipe.prepare(t)
    args = (pipe.nodes_t, pipe.edges_t, pipe.ew_t, f.tpos, f.conf, f.src, f.anchors, f.weights, f.tgt, pipe.intr)
    r = ref.optimize(*args, prev_rot=prev_r, prev_trans=prev_t)
    row = {"frame": t}
    for name, s in solvers.items():
        o = s.optimize(*args, prev_rot=prev_r, prev_trans=prev_t)
        row[name] = dict(dt=(o["node_translations"] - r["node_translations"]).abs().max().item(),
                         dr=(o["node_rotations"] - r["node_rotations"]).abs().max().item(),
                         iters=o["convergence_info"]["pcg_iterations"],
                         per_step=[int(x) for x in s.stats()[:, 0]])
    prev_r, prev_t = r["node_rotations"], r["node_translations"]
    res.append(row)
    print(json.dumps(row), flush=True)
