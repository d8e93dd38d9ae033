"""Tuning tool (CPU, not product): node count of each BASELINE config's depth-mesh graph for a node coverage,
built by the reference's own compiled C++ (oracle/_ref: backproject_depth_float, compute_mesh_from_depth,
erode_mesh, sample_nodes, compute_edges_geodesic, node_and_edge_clean_up) on the config's source frame — the
numbers behind BASELINE_CONFIGS[c]["coverage"] in occlusionfusion_amd/synthetic.py.

  python tools/graph_coverage.py [config coverage ...]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
from occlusionfusion_amd import synthetic as S  # noqa: E402
from make_golden import csrc_depth_graph  # noqa: E402


def main():
    args = sys.argv[1:]
    pairs = ([(int(args[i]), float(args[i + 1])) for i in range(0, len(args), 2)] if args else
             [(c, S.BASELINE_CONFIGS[c]["coverage"]) for c in (1, 2, 3, 4)])
    for cfg, cov in pairs:
        c = S.BASELINE_CONFIGS[cfg]
        scene, seed = S.config_scene(cfg)
        cam = S.bench_camera(c["cam_scale"])
        t0 = time.time()
        nodes, edges, _ = csrc_depth_graph(S.source_depth(scene, cam, seed), cam, cov)
        print(f"config {cfg} coverage {cov}: {nodes.shape[0]} nodes, {(edges >= 0).sum()} edges "
              f"({time.time() - t0:.1f} s)", flush=True)


if __name__ == "__main__":
    main()
