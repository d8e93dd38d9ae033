"""Tuning study (GPU, not product): the GN transforms' max error against every f64 oracle fixture, and the PCG
iterations, for several PCG stop settings — the GPU counterpart of tools/stoprule_study.py.

    python tools/gn_tol_errors.py [pcg_tol ...]      (default 1e-6 2e-6 3e-6; pcg_err_tol stays the default)
Prints one JSON line per (fixture, pcg_tol): max |dR|, max |dt|, the loss log's max relative error, PCG iterations.
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
from occlusionfusion_amd import GaussNewtonSolver  # noqa: E402
from test_gpu_golden_gn import _load, _frame, _problem  # noqa: E402
from test_gpu_moose import _cam  # noqa: E402

dev = torch.device("cuda", 0)


def err(out, R, t, loss):
    dr = float(np.abs(out["node_rotations"].cpu().numpy() - R).max())
    dt = float(np.abs(out["node_translations"].cpu().numpy() - t).max())
    tot = np.asarray(out["convergence_info"]["total"], np.float64)
    lr = float(np.abs(tot / loss[:len(tot)] - 1).max()) if len(tot) == len(loss) else float("nan")
    return dr, dt, lr, int(out["_status"][2].item())


def chain(name, tol, n=None):
    g = _load(name + ".npz")
    N = g["nodes"].shape[0]
    s = GaussNewtonSolver(N, 10000, pcg_tol=tol)
    intr = tuple(float(v) for v in g["intr"])
    R = T = None
    res = []
    for q in range(n or len(g["frames"])):
        out = s.optimize(**_problem(g, _frame(g, q, dev), dev), intrinsics=intr, prev_rot=R, prev_trans=T)
        R, T = out["node_rotations"], out["node_translations"]
        res.append((f"{name}:{q}",) + err(out, g[f"f{q}_R"], g[f"f{q}_t"], g[f"f{q}_loss_total"]))
    return res


def single(name, tol):
    g = _load(name + ".npz")
    N = g["nodes"].shape[0]
    s = GaussNewtonSolver(N, 10000, pcg_tol=tol)
    if name == "moose":
        out = s.optimize(g["nodes"], g["edges"], g["edge_weights"], g["nodes"], np.zeros(N, np.float32), g["src"],
                         g["anchors"], g["weights"], g["tgt"], _cam(g).as_vec())
    else:
        out = s.optimize(g["nodes"], g["edges"], g["edge_weights"], g["tpos"], g["conf"], g["src"], g["anchors"],
                         g["weights"], g["tgt"], tuple(float(v) for v in g["intr"]))
    return [(name,) + err(out, g["R"], g["t"], g["loss_total"])]


tols = [float(v) for v in sys.argv[1:]] or [1e-6, 2e-6, 3e-6]
for tol in tols:
    rows = chain("gn_2k", tol) + chain("gn_4k", tol) + chain("gn_c5r1", tol) + chain("gn_c5r7", tol) + \
        single("gn_1k", tol) + single("moose", tol)
    for r in rows:
        print(json.dumps({"pcg_tol": tol, "fixture": r[0], "dR": r[1], "dt": r[2], "loss_rel": r[3], "pcg": r[4]}))
    print(json.dumps({"pcg_tol": tol, "max_dR": max(r[1] for r in rows), "max_dt": max(r[2] for r in rows),
                      "max_loss_rel": max(r[3] for r in rows), "pcg_total": sum(r[4] for r in rows)}), flush=True)
