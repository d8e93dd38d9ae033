"""Tuning study (not product): the moose pair's PCG work and accuracy against the preconditioner refresh threshold
(precond_rot_tol) under both preconditioners."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
import torch  # noqa: F401

from test_gpu_moose import _moose_gn

g = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "moose.npz"),
            allow_pickle=False)
for pc in ("schwarz", "cluster"):
    for tol in (0.1, 0.2, 0.3, 0.5, 0.0):
        out, dr, dt = _moose_gn(g, precond=pc, precond_rot_tol=tol)
        ci = out["convergence_info"]
        print(f"{pc:8s} precond_rot_tol {tol:4.2f}: PCG iterations {ci['pcg_iterations']:6d}, capped {ci['pcg_capped_steps']}, "
              f"max error {max(dr, dt):.3g}", flush=True)
