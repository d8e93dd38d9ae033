"""Moose landmark GN: transform / loss error against the dense f64 oracle fixture at several PCG stop settings
(relative residual pcg_tol, error-based pcg_err_tol; 0 = residual alone)."""
import os
import sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from occlusionfusion_amd import GaussNewtonSolver  # noqa: E402

g = np.load("tests/golden/moose.npz", allow_pickle=False)
N = g["nodes"].shape[0]
K = g["K"]
for tol, et in ((1e-6, 0.0), (1e-8, 0.0), (1e-6, 1e-5), (1e-6, 3e-6), (1e-6, 3e-5)):
    s = GaussNewtonSolver(N, 1000, pcg_tol=tol, pcg_err_tol=et)
    out = s.optimize(g["nodes"], g["edges"], g["edge_weights"], g["nodes"], np.zeros(N, np.float32), g["src"],
                     g["anchors"], g["weights"], g["tgt"], np.array([K[0, 0], K[1, 1], K[0, 2], K[1, 2]]))
    dr = np.abs(out["node_rotations"].cpu().numpy() - g["R"]).max()
    dt = np.abs(out["node_translations"].cpu().numpy() - g["t"]).max()
    lr = np.abs(np.array(out["convergence_info"]["total"]) / g["loss_total"] - 1).max()
    print(f"tol {tol:g} err_tol {et:g}: dR {dr:.3g} dt {dt:.3g} loss rel {lr:.3g} pcg {out['convergence_info']['pcg_iterations']} per step {s.stats()[:, 0].astype(int).tolist()}",
          flush=True)
