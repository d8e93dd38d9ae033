"""Tuning probe (not product): how many of the warped integrate's listed bricks update no voxel (the ceiling of a
brick-level cull), and how many skin-valid voxels they hold, on the bench's config-3 frames."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from occlusionfusion_amd import synthetic as S
    from occlusionfusion_amd.pipeline import FusionPipeline
    dev = torch.device("cuda", 0)
    cfg = S.BASELINE_CONFIGS[3]
    seq = S.config_sequence(3, device=dev)
    D = cfg["dims"]
    pipe = FusionPipeline(seq, cfg["origin"], cfg["voxel"], (D, D, D), device=dev)
    frames = [pipe.prepare(t) for t in range(12)]
    pipe.integrate_source(frames[0])
    cache = pipe.wf.skin_tsdf_cache()
    K = cache.k
    valid = (cache.anchors.view(-1, 4)[:, K - 1] != -1).view(cache.n_list, 512) if cache.n_list else None
    nvalid = valid.sum(1).cpu().numpy()
    out = []
    for t in range(1, 11):
        pipe.solve(frames[t], None)
        pipe.integrate(frames[t], t, count_updates=True)
        torch.cuda.synchronize()
        cnt = pipe.vol.n_updated[:cache.n_list].cpu().numpy()
        zero = cnt == 0
        out.append({"frame": t, "listed": int(cache.n_list), "zero_update_bricks": int(zero.sum()),
                    "skin_valid_voxels_in_them": int(nvalid[zero].sum()), "skin_valid_voxels": int(nvalid.sum()),
                    "updated": int(cnt.sum())})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
