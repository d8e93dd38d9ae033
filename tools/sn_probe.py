import sys, os, time
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np, torch
sys.path.insert(0, "tests")
dev = torch.device("cuda", 0)
from occlusionfusion_amd.graph_proc import MeshGraph
from occlusionfusion_amd.image_proc import compute_mesh_from_depth_device
rng = np.random.default_rng(4)
H = W = 512
yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
z = (1.2 + 0.1 * np.sin(xx / 40) * np.cos(yy / 55) + rng.normal(0, 0.0005, (H, W))).astype(np.float32)
P = np.stack([(xx - 256) * z / 500, (yy - 256) * z / 500, z]).astype(np.float32)
m = compute_mesh_from_depth_device(torch.from_numpy(P).to(dev), 0.05)
mg = MeshGraph(m["vertices"], m["faces"], dev)
ne = mg.erode(1, 3)
for cov in (0.05, 0.02):
    for r in range(3):
        torch.cuda.synchronize(); t = time.perf_counter()
        pos, idx = mg.sample_nodes(ne, cov)
        torch.cuda.synchronize()
        print(cov, "nodes", idx.shape[0], "ms", 1e3 * (time.perf_counter() - t), flush=True)
