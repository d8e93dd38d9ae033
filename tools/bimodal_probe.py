"""Is the per-run PCG launch-time spread (~5.0 vs ~5.3 us) a property of the process or of
the allocation? One process: two pipelines (separate allocations), each timed over 3 back-to-back windows of
30 config-3 frames; prints us per PCG launch per window. Not part of the bench."""
import sys, time
import torch
sys.path.insert(0, ".")
from occlusionfusion_amd import synthetic as S
from occlusionfusion_amd.pipeline import FusionPipeline

c = S.BASELINE_CONFIGS[3]
seq = S.config_sequence(3)
dev = torch.device("cuda:0")
for p in range(2):
    pipe = FusionPipeline(seq, c["origin"], c["voxel"], (c["dims"],) * 3, n_matches=10000, device=dev)
    frames = [pipe.prepare(t) for t in range(95)]
    torch.cuda.synchronize()
    pipe.integrate_source(frames[0])
    t = 1
    for w in range(3):
        pipe.solver.timing(True)
        t0 = time.perf_counter()
        for _ in range(30):
            pipe.solve(frames[t], frames[t + 1])
            pipe.integrate(frames[t], t)
            t += 1
        pipe.solver.drain()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        ms, n, _ = pipe.solver.timing(False)
        print(f"pipeline {p} window {w}: {1e3 * ms / max(n, 1):.3f} us per PCG launch, {30 / el:.1f} frames/s",
              flush=True)
    del pipe, frames
    torch.cuda.empty_cache()
