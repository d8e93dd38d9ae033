"""GPU diagnostic (round 6): where the one-launch Schwarz iteration (k_as_iter) and the two-launch form
(OFX_AS_ONE=0) part. One GN step with the PCG capped at k iterations, both forms, k = 1..K; also under the tuning
overrides OFX_PCG_W1=1 (one wave per cluster in the two-launch form) and OFX_PCG_KU=<n>.
Usage: python tools/one_launch_diag.py gn_4k.npz [K] [ENV=VAL ...]"""
import os
import sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np
import torch

name = sys.argv[1]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 6
for kv in sys.argv[3:]:
    k_, v_ = kv.split("=")
    os.environ[k_] = v_
from occlusionfusion_amd import GaussNewtonSolver  # noqa: E402

g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", name), allow_pickle=False)
p = "f0_" if "frames" in g.files else ""
os.environ["OFX_PRECOND"] = "as"


def run(one, k, steps=1):
    os.environ["OFX_AS_ONE"] = str(one)
    s = GaussNewtonSolver(g["nodes"].shape[0], 10000, num_iter=steps, pcg_max_iter=k)
    out = s.optimize(g["nodes"], g["edges"], g["edge_weights"], g[p + "tpos"], g[p + "conf"], g[p + "src"],
                     g[p + "anchors"], g[p + "weights"], g[p + "tgt"], tuple(float(v) for v in g["intr"]))
    torch.cuda.synchronize()
    return out["node_rotations"].cpu().numpy(), out["node_translations"].cpu().numpy(), s.precond_info()


for k in list(range(1, K + 1)) + [2000]:
    a, b = run(0, k), run(1, k)
    print(f"pcg_max_iter {k:5d}: launches/it {a[2]['launches_per_iteration']}/{b[2]['launches_per_iteration']} "
          f"max|dR| {np.abs(a[0] - b[0]).max():.3e} max|dt| {np.abs(a[1] - b[1]).max():.3e} "
          f"equal {np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])}", flush=True)

if os.environ.get("DIAG_NODES"):
    k = int(os.environ["DIAG_NODES"])
    a, b = run(0, k), run(1, k)
    os.environ["OFX_AS_ONE"] = "1"
    s = GaussNewtonSolver(g["nodes"].shape[0], 10000, num_iter=1, pcg_max_iter=k)
    s.optimize(g["nodes"], g["edges"], g["edge_weights"], g[p + "tpos"], g[p + "conf"], g[p + "src"],
               g[p + "anchors"], g[p + "weights"], g[p + "tgt"], tuple(float(v) for v in g["intr"]))
    perm = s.row_order()
    row_of = {int(n): r for r, n in enumerate(perm) if n >= 0}
    d = np.maximum(np.abs(a[1] - b[1]).max(1), np.abs(a[0] - b[0]).reshape(a[0].shape[0], -1).max(1))
    bad = np.nonzero(d > 0)[0]
    print(f"k={k}: {bad.size} of {d.size} nodes differ; rows {len(perm)}")
    top = np.argsort(-d)[:25]
    print("top nodes (node, row, cluster, diff):", [(int(n), row_of[int(n)], row_of[int(n)] // 8, float(f"{d[n]:.2e}"))
                                                   for n in top])
    cl = np.bincount([row_of[int(n)] // 8 for n in bad], minlength=len(perm) // 8)
    print("clusters with differing nodes:", np.nonzero(cl)[0].tolist()[:80])
