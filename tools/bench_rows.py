"""Measurement of the SURVEY §8(f) rows on the bench scene (512³ @4 mm after the source frame and a few warped
frames, 640x448 depth) — one JSON object, written to --out (profiles/r01_rows.json).

Per op: median of --reps timed calls (torch events on the stream libofx is called on; ops that size their
output synchronise inside, which the timing includes), plus for the byte-streaming kernels the algorithmic
bytes and GB/s against the 8 TB/s HBM peak. CPU datapoints: the REFERENCE's own compiled C++ (oracle/_ref,
csrc image_proc / graph_proc, OpenMP where the reference uses it) on the same inputs, on this host.

  python tools/bench_rows.py [--dims 512] [--nodes 2000] [--reps 5] [--out profiles/r01_rows.json]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

PEAK = 8.0e12


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        out = fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e-3)
    return float(np.median(ts)), out


def host_timed(fn, reps=3):
    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--dims", type=int, default=512)
    p.add_argument("--voxel", type=float, default=0.004)
    p.add_argument("--nodes", type=int, default=2000)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--frames", type=int, default=4)
    p.add_argument("--out", default=None)
    p.add_argument("--no-cpu", action="store_true")
    a = p.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from occlusionfusion_amd import EDGraph
    from occlusionfusion_amd import synthetic as S
    from occlusionfusion_amd.graph_proc import MeshGraph, clusters_device, knn_device, node_edge_cleanup_device
    from occlusionfusion_amd.graph_proc import pixel_anchors_euclidean_device
    from occlusionfusion_amd.image_proc import (backproject_depth_device, compute_mesh_from_depth_device,
                                                depth_2_pc_device)
    from occlusionfusion_amd.pipeline import FusionPipeline

    D = a.dims
    seq = S.SyntheticSequence.build(a.nodes, seed=3)
    pipe = FusionPipeline(seq, (-D * a.voxel / 2, -D * a.voxel / 2, 0.5), a.voxel, (D, D, D), device=dev)
    frames = [pipe.prepare(t) for t in range(a.frames + 1)]
    pipe.integrate_source(frames[0])
    for t in range(1, a.frames + 1):
        pipe.step(frames[t], t)
    torch.cuda.synchronize()
    vol, cam = pipe.vol, seq.cam
    V = D ** 3
    rows = {"workload": f"{D}^3 TSDF @{a.voxel * 1e3:g} mm after {a.frames} fused frames; 640x448 depth; "
                        f"{seq.nodes.shape[0]} nodes", "reps": a.reps}

    # ---- a7: source-frame integrate (the dense pass, once per sequence) on a scratch volume of the same grid
    from occlusionfusion_amd import TSDFVolume
    scratch = TSDFVolume.from_grid(vol._vol_origin, vol._voxel_size, vol._vol_dim, pipe.intr, pipe.fopt, device=dev)

    def src_pass():
        if hasattr(scratch, "frame_id"):
            del scratch.frame_id
        scratch.update(frames[0].im, 0)
        scratch.integrate_device(count_updates=True)
    t_src, _ = timed(src_pass, a.reps)
    U_src = int(scratch.n_updated[:scratch.n_bricks].sum().item())
    B_src = V * 8 + U_src * 16
    rows["a7_source_frame_integrate"] = {"ms": 1e3 * t_src, "updated_voxels": U_src, "bytes": B_src,
                                         "GBps": B_src / t_src / 1e9, "frac_hbm": B_src / t_src / PEAK,
                                         "bytes_note": "tsdf + weight read 8 B per voxel, tsdf/weight/colour "
                                                       "write + colour read 16 B per updated voxel (SURVEY 8(d))"}
    del scratch
    # ---- new capability: raycast of the fused volume (no reference twin)
    t_rc, rc = timed(lambda: vol.raycast(), a.reps)
    rows["new_raycast"] = {"ms": 1e3 * t_rc, "pixels": int(rc[0].numel()), "hits": int((rc[0] > 0).sum().item()),
                           "note": "depth + normals + colours, trilinear march (coarse 0.8 trunc / fine 1 voxel)"}

    # ---- f1: surface extraction
    t_tr, _ = timed(lambda: vol.truncated_region_device(1.2), a.reps)
    B_tr = vol.n_slots * (4 + 1)
    rows["f1_truncated_region"] = {"ms": 1e3 * t_tr, "bytes": B_tr, "GBps": B_tr / t_tr / 1e9,
                                   "frac_hbm": B_tr / t_tr / PEAK,
                                   "bytes_note": "tsdf read 4 B + mask write 1 B per voxel slot"}
    t_mc, m = timed(lambda: vol.extract_mesh_device(use_mask=True, max_diff=1.2), a.reps)
    t_mesh, mesh = timed(lambda: vol.get_mesh(), a.reps)
    rows["f1_marching_cubes"] = {"ms": 1e3 * t_mc, "verts": int(m["verts"].shape[0]), "faces": int(m["faces"].shape[0]),
                                 "note": "masked MC incl. truncated region, count (1 sync) + emit + normals"}
    rows["f1_get_mesh"] = {"ms": 1e3 * t_mesh, "note": "get_mesh incl. world coordinates, colours, D2H copies"}
    # sharded marching cubes: 4 slab shards of the same volume in one process (halo columns sliced from the
    # neighbours, as exchange_boundary delivers them), per-shard meshing + key merge
    from occlusionfusion_amd import TSDFVolume
    from occlusionfusion_amd.sharding import merge_shard_meshes
    W4 = 4
    col = vol.brick_column_slots()
    shards = []
    for r in range(W4):
        sh = TSDFVolume.from_grid(vol._vol_origin, vol._voxel_size, vol._vol_dim, (cam.fx, cam.fy, cam.cx, cam.cy),
                                  device=dev, shard=(r, W4))
        sh.tsdf_b.copy_(vol.tsdf_b[col * sh.brick_x0: col * sh.brick_x1])
        sh.color_b.copy_(vol.color_b[col * sh.brick_x0: col * sh.brick_x1])
        shards.append(sh)
    bnd = [sh.boundary_columns() for sh in shards]
    t_part = []

    def sharded():
        parts = []
        for r, sh in enumerate(shards):
            parts.append(sh.extract_mesh_shard(bnd[r - 1][1] if r > 0 else None, bnd[r + 1][0] if r < W4 - 1 else None))
        return merge_shard_meshes(parts, vol._vol_dim)
    t_sh, msh = timed(sharded, a.reps)
    t_one, _ = timed(lambda: shards[1].extract_mesh_shard(bnd[0][1], bnd[2][0]), a.reps)
    rows["f1_marching_cubes_sharded"] = {"shards": W4, "ms_all_shards_sequential_plus_merge": 1e3 * t_sh,
                                         "ms_one_shard": 1e3 * t_one, "verts": int(msh["verts"].shape[0]),
                                         "equal_to_whole": bool(msh["verts"].shape[0] == m["verts"].shape[0]),
                                         "note": "one process; per rank a shard costs ms_one_shard + the halo "
                                                 "exchange + gather"}
    del shards, bnd

    # ---- f3: correspondence front-end
    depth = frames[-1].im[5].contiguous()
    H, W = depth.shape
    t_bp, P = timed(lambda: backproject_depth_device(depth, cam.fx, cam.fy, cam.cx, cam.cy), a.reps)
    B_bp = H * W * (4 + 12)
    rows["f3_backproject"] = {"ms": 1e3 * t_bp, "GBps": B_bp / t_bp / 1e9, "frac_hbm": B_bp / t_bp / PEAK}
    t_dm, dm = timed(lambda: compute_mesh_from_depth_device(P, 0.05), a.reps)
    rows["f3_depth_mesh"] = {"ms": 1e3 * t_dm, "verts": int(dm["vertices"].shape[0]), "faces": int(dm["faces"].shape[0])}
    K = np.array([[cam.fx, 0, cam.cx], [0, cam.fy, cam.cy], [0, 0, 1.0]])
    t_pc, _ = timed(lambda: depth_2_pc_device(depth, K), a.reps)
    rows["f3_target_point_cloud"] = {"ms": 1e3 * t_pc, "note": "depth_2_pc + compaction + pixel map (1 sync: count)"}

    # ---- f2: standalone skinning on the canonical mesh / image
    verts = torch.from_numpy(mesh[0]).to(dev)
    t_sk, _ = timed(lambda: pipe.wf.skin_device(verts), a.reps)
    rows["f2_skin_mesh"] = {"ms": 1e3 * t_sk, "points": int(verts.shape[0]), "nodes": int(seq.nodes.shape[0])}
    nodes_t = pipe.nodes_t
    t_pa, _ = timed(lambda: pixel_anchors_euclidean_device(nodes_t, P, seq.node_coverage), a.reps)
    rows["f2_pixel_anchors_euclidean"] = {"ms": 1e3 * t_pa, "pixels": H * W}
    t_kn, _ = timed(lambda: knn_device(verts, nodes_t, 1), a.reps)
    rows["f2_knn1_mesh"] = {"ms": 1e3 * t_kn}

    # ---- f4: graph construction from the canonical mesh
    faces = torch.from_numpy(mesh[1].astype(np.int32)).to(dev)
    t_gc, mg = timed(lambda: MeshGraph(verts, faces, dev), a.reps)
    t_er, ne = timed(lambda: mg.erode(1, 3), a.reps)
    t_sn, (pos, idx) = timed(lambda: mg.sample_nodes(ne, 0.05), a.reps)
    t_geo, (E, Wt, Dd, _) = timed(lambda: mg.edges_geodesic(idx, 8, 0.05), a.reps)
    t_cu, _ = timed(lambda: node_edge_cleanup_device(E, torch.ones(E.shape[0], dtype=torch.bool, device=dev)), a.reps)
    t_cl, _ = timed(lambda: clusters_device(E), a.reps)
    t_all, gr = timed(lambda: EDGraph.from_mesh(mesh[0], mesh[1], {"node_coverage": 0.05}, device=dev), a.reps)
    from occlusionfusion_amd.graph_proc import downsample_device
    t_ds, (dsd, _) = timed(lambda: downsample_device(pos, 0.1, dev), a.reps)
    rows["f4_pyramid_downsample"] = {"ms": 1e3 * t_ds, "nodes_in": int(pos.shape[0]), "kept": len(dsd)}
    rows["f4_graph"] = {"mesh_verts": int(verts.shape[0]), "mesh_faces": int(faces.shape[0]),
                        "nodes": int(idx.shape[0]), "sample_rounds": int(mg.sample_rounds),
                        "ms_adjacency": 1e3 * t_gc, "ms_erode": 1e3 * t_er, "ms_sample_nodes": 1e3 * t_sn,
                        "ms_edges_geodesic": 1e3 * t_geo, "geodesic_sequential_nodes": int(mg.geodesic_sequential), "ms_cleanup": 1e3 * t_cu, "ms_clusters": 1e3 * t_cl,
                        "ms_from_mesh_total": 1e3 * t_all, "nodes_after_cleanup": int(gr.nodes.shape[0])}

    # ---- CPU: the reference's compiled C++ on the same inputs (this host)
    if not a.no_cpu:
        from oracle.build_ref import load_prebuilt
        m = load_prebuilt()
        if m is None:
            rows["cpu_reference"] = None
        else:
            dn = depth.cpu().numpy()
            Pn = P.cpu().numpy()
            vn, fn = mesh[0].astype(np.float32), mesh[1].astype(np.int32)
            cpu = {"threads": int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))}
            out = np.zeros((3, H, W), np.float32)
            cpu["f3_backproject_ms"] = 1e3 * host_timed(
                lambda: m.backproject_depth_float(dn, out, cam.fx, cam.fy, cam.cx, cam.cy))

            def dmesh():
                v, px, f = np.zeros((0,), np.float32), np.zeros((0,), np.int32), np.zeros((0,), np.int32)
                m.compute_mesh_from_depth(Pn, 0.05, v, px, f)
            cpu["f3_depth_mesh_ms"] = 1e3 * host_timed(dmesh)
            nn = seq.nodes.astype(np.float32)

            def panc():
                pa, pw = np.zeros((0,), np.int32), np.zeros((0,), np.float32)
                m.compute_pixel_anchors_euclidean(nn, Pn, float(seq.node_coverage), pa, pw)
            cpu["f2_pixel_anchors_euclidean_ms"] = 1e3 * host_timed(panc, 1)
            t0 = time.perf_counter()
            ne_c = m.erode_mesh(vn, fn, 1, 3)
            cpu["f4_erode_ms"] = 1e3 * (time.perf_counter() - t0)
            npos, nidx = np.zeros((0,), np.float32), np.zeros((0,), np.int32)
            t0 = time.perf_counter()
            n = m.sample_nodes(vn, ne_c, npos, nidx, 0.05, True, False)
            cpu["f4_sample_nodes_ms"] = 1e3 * (time.perf_counter() - t0)
            E_c = -np.ones((n, 8), np.int32)
            W_c, D_c = np.zeros((n, 8), np.float32), np.zeros((n, 8), np.float32)
            n2v = -np.ones((n, vn.shape[0]), np.float32)
            t0 = time.perf_counter()
            m.compute_edges_geodesic(vn, np.ones((vn.shape[0], 1), bool), fn, nidx[:n], 8, 0.05, E_c, W_c, D_c, n2v,
                                     True, True)
            cpu["f4_edges_geodesic_ms"] = 1e3 * (time.perf_counter() - t0)
            cpu["f4_nodes"] = int(n)
            cpu["f4_equal_to_gpu"] = bool(n == idx.shape[0] and np.array_equal(nidx[:n, 0], idx.cpu().numpy())
                                          and np.array_equal(E_c, E.cpu().numpy()))
            rows["cpu_reference"] = cpu
    line = json.dumps(rows)
    print(line, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
