"""Tuning/debug probe: repeat the parallel geodesic edges on the 512² noisy depth mesh and compare every run
with the sequential heap kernel (OFX_GEO_SEQ=1): reports differing nodes and the per-run sequential counts."""
import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
sys.path.insert(0, "tests")
import numpy as np, torch
from test_gpu_graph import _noisy_depth_mesh
dev = torch.device("cuda", 0)
m, mg = _noisy_depth_mesh(dev)
ne = mg.erode(1, 3)
_, idx = mg.sample_nodes(ne, 0.05)
os.environ["OFX_GEO_SEQ"] = "1"
Es, Ws, Ds, _ = mg.edges_geodesic(idx, 8, 0.05)
del os.environ["OFX_GEO_SEQ"]
for r in range(6):
    if r >= 3:
        os.environ["OFX_GEO_BIG"] = "1"   # runs 3-5: the 16384-slot form for every node
    E, W, D, _ = mg.edges_geodesic(idx, 8, 0.05)
    bad = torch.nonzero((E != Es).any(1) | (D != Ds).any(1)).reshape(-1).tolist()
    print("run", r, "sequential nodes", mg.geodesic_sequential, "differing nodes", bad[:10], flush=True)
    for n in bad[:3]:
        print("  node", n, "par E", E[n].tolist(), "D", D[n].tolist())
        print("  node", n, "seq E", Es[n].tolist(), "D", Ds[n].tolist())
