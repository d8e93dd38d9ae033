"""PCG iterations per GN step over a bench-like frame loop (config 3 by default), for the chunk-sizing study of the PCG
host loop (drained launches). Writes gpurun_out/pcg_counts_c<config>.json: per frame the 10 per-step counts.
Usage: python tools/pcg_counts.py [config] [frames]
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
from occlusionfusion_amd import synthetic as S  # noqa: E402
from occlusionfusion_amd.pipeline import FusionPipeline  # noqa: E402

cfg_i = int(sys.argv[1]) if len(sys.argv) > 1 else 3
n = int(sys.argv[2]) if len(sys.argv) > 2 else 120
cfg = S.BASELINE_CONFIGS[cfg_i]
dev = torch.device("cuda", 0)
seq = S.config_sequence(cfg_i, cfg["nodes"], rank=0, device=dev)
D = cfg["dims"]
pipe = FusionPipeline(seq, cfg["origin"], cfg["voxel"], (D, D, D), n_matches=10000, device=dev)
frames = [pipe.prepare(t) for t in range(n + 2)]
pipe.integrate_source(frames[0])
rows = []
for t in range(1, n + 1):
    pipe.solve(frames[t], frames[t + 1])
    pipe.integrate(frames[t], t)
    torch.cuda.synchronize()
    st = pipe.solver.stats()
    rows.append([int(v) for v in st[:, 0]])
    if t % 20 == 0:
        print(t, rows[-1], flush=True)
os.makedirs("gpurun_out", exist_ok=True)
with open(f"gpurun_out/pcg_counts_c{cfg_i}.json", "w") as f:
    json.dump({"config": cfg_i, "nodes": int(seq.nodes.shape[0]), "counts": rows}, f)
print("mean per frame", sum(map(sum, rows)) / len(rows))
