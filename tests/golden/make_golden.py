"""Generate the committed golden fixtures in tests/golden/ (run in the CPU build container).

  skin_csrc.npz       — skinning k-NN vectors produced by the REFERENCE's own compiled C++
                        (csrc compute_pixel_anchors_euclidean / sample_nodes / compute_edges_euclidean,
                        built from /root/reference by oracle/build_ref.py) + the oracle's skin of the
                        same points. Pins the oracle's k-NN to the reference.
  integrate_small.npz — a 66x52x70 volume fused over a source frame and one ED-warped frame by the
                        oracle restatement of tsdf.py/warpfield.py/geometry.py (inputs + expected
                        tsdf/weight/colour + skin valid mask).
  anchors_csrc.npz    — compute_pixel_anchors_euclidean / _geodesic and update_pixel_anchors outputs of the
                        REFERENCE's compiled C++ (csrc/cpu/graph_proc.cpp:483-709,934-961): a point image with
                        duplicated nodes (distance ties) and a node->vertex distance matrix with ties and -1s.
  graph_csrc.npz      — ED-graph construction by the REFERENCE's compiled C++ (graph_proc.cpp:17-481) on two
                        meshes (a depth mesh of the synthetic frame and an exact grid plane, whose equal edge
                        lengths tie the Dijkstra priority queue): erode_mesh, sample_nodes (no shuffle),
                        compute_edges_geodesic in the three modes EDGraph uses, node_and_edge_clean_up,
                        compute_clusters, compute_edges_euclidean.
  gn_small.npz        — one DeformNet.optimize solve (N≈100, M=600) by the dense f64 oracle.
  gn_1k.npz           — one DeformNet.optimize solve at BASELINE config 2's size (rigid sequence, 1025 nodes,
                        10k matches, dense J ≈ 57k x 6k) by the dense f64 oracle (≈2 min on 8 cores).
  gn_2k.npz           — the headline config's solve (config 3: occluded non-rigid frames 10 and 11, the second
                        chained from the first, ~2k nodes of the SURVEY §8(d) depth-mesh graph built by the
                        reference's C++, 10k matches) by the f64 oracle with a sparse JᵀJ + dense LU.
  gn_4k.npz           — the same at config 4's graph (~4k nodes, frame 10).
  gn_2k_hole.npz      — gn_2k's frame 10 with the matches of a 48-node patch removed (the patch held only by ARAP and
                        confidence-0.3 motion rows): a differently conditioned spectrum for the PCG stop rule.
  gn_c5r1.npz,        — BASELINE config 5 (one independent 512³ scene per GPU): the scenes of ranks 1 and 7
  gn_c5r7.npz           (synthetic.config_scene(5, r): their own sphere, occluder and motion phase), frame 10, the
                        same solve at their own ~2k-node depth-mesh graphs.
  frontend_csrc.npz   — backproject_depth_float / _ushort and compute_mesh_from_depth outputs of the
                        REFERENCE's compiled C++ (csrc/cpu/image_proc.cpp:351-545) on a synthetic frame,
                        incl. max-distance thresholds that tie exactly with triangle edge lengths; plus the
                        oracle's depth_2_pc target cloud (geometry.py:44-59) of the same frame.

Usage: python tests/golden/make_golden.py [which ...]  (e.g. gn5)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import fusion_oracle as fo  # noqa: E402
from occlusionfusion_amd import synthetic as S  # noqa: E402


def small_setup(seed=11):
    cam = S.Intrinsics(525.0 / 4, 525.0 / 4, 319.5 / 4, (239.5 - 16) / 4, 160, 112)
    scene = S.SphereScene()
    rng = np.random.default_rng(seed)
    d0 = scene.render(cam, 0, rng)
    d1 = scene.render(cam, 1, rng)
    pts = S.backproject(d0, cam)
    nodes = S.sample_nodes(pts, 0.07, seed)
    edges, ew = S.euclidean_edges(nodes, 8)
    return cam, scene, d0, d1, pts, nodes, edges, ew


def small_transforms(scene, nodes, t, seed):
    rng = np.random.default_rng(seed)
    N = nodes.shape[0]
    aa = rng.normal(0, 0.02, (N, 3))
    R = fo.angle_axis_to_rotation_matrix(aa).astype(np.float32)
    T = (scene.deform_points(nodes, t) - nodes + rng.normal(0, 0.002, (N, 3))).astype(np.float32)
    return R, T


def make_skin_csrc():
    from oracle.build_ref import build
    m = build()
    rng = np.random.default_rng(5)
    surf = rng.normal(size=(4000, 3))
    surf = 0.3 * surf / np.linalg.norm(surf, axis=1, keepdims=True) + np.array([0, 0, 1.4])
    surf = surf.astype(np.float32)
    npos = np.zeros((0, 3), np.float32)
    nidx = np.zeros((0, 1), np.int32)
    n = m.sample_nodes(surf, np.ones((surf.shape[0], 1), bool), npos, nidx, 0.05, False, False)
    nodes = np.ascontiguousarray(npos[:n])
    edges = m.compute_edges_euclidean(nodes, 8)
    q = (surf[rng.choice(surf.shape[0], 3000)] + rng.normal(0, 0.05, (3000, 3))).astype(np.float32)
    img = np.ascontiguousarray(q.T.reshape(3, 1, -1))
    pa = np.zeros((0,), np.int32)
    pw = np.zeros((0,), np.float32)
    m.compute_pixel_anchors_euclidean(nodes, img, 0.05, pa, pw)
    oa, ow, ov = fo.skin(q, nodes, 0.05)
    np.savez_compressed(os.path.join(HERE, "skin_csrc.npz"), points=q, nodes=nodes, node_coverage=0.05,
                        csrc_edges=edges, csrc_anchors=pa.reshape(-1, 4), csrc_weights=pw.reshape(-1, 4),
                        oracle_anchors=oa, oracle_weights=ow, oracle_valid=ov)
    print("skin_csrc:", nodes.shape[0], "nodes,", q.shape[0], "points")


def make_frontend_csrc():
    from oracle.build_ref import build
    m = build()
    cam, scene, d0, d1, pts, nodes, edges, ew = small_setup()
    rng = np.random.default_rng(3)
    depth = d1.astype(np.float32)
    depth_u16 = np.round(depth * 1000.0).astype(np.uint16)
    intr = np.array([cam.fx, cam.fy, cam.cx, cam.cy], np.float32)
    bf = np.zeros((3,) + depth.shape, np.float32)
    m.backproject_depth_float(depth, bf, *[float(v) for v in intr])
    bu = np.zeros((3,) + depth.shape, np.float32)
    m.backproject_depth_ushort(depth_u16, bu, *[float(v) for v in intr], 1000.0)
    # thresholds: the reference default (0.05), a tight one, and exact ties with realised edge lengths
    xs = bf[:, :-1, :-1].reshape(3, -1).T
    nb = bf[:, 1:, :-1].reshape(3, -1).T
    ok = (xs[:, 2] > 0) & (nb[:, 2] > 0)
    lens = np.array([fo._edge_len_f32(a, b) for a, b in zip(xs[ok][:4000], nb[ok][:4000])], np.float32)
    ties = np.sort(rng.choice(lens, 2, replace=False))
    thresholds = np.array([0.05, np.median(lens) * 1.01, ties[0], ties[1]], np.float32)
    meshes = {}
    for i, t in enumerate(thresholds):
        v = np.zeros((0,), np.float32)
        px = np.zeros((0,), np.int32)
        f = np.zeros((0,), np.int32)
        m.compute_mesh_from_depth(bf, float(t), v, px, f)
        meshes[f"mesh{i}_vertices"] = v.reshape(-1, 3)
        meshes[f"mesh{i}_pixels"] = px.reshape(-1, 2)
        meshes[f"mesh{i}_faces"] = f.reshape(-1, 3)
    K = np.eye(3)
    K[0, 0], K[1, 1], K[0, 2], K[1, 2] = intr
    pc, pmap = fo.target_point_cloud(depth, K)
    np.savez_compressed(os.path.join(HERE, "frontend_csrc.npz"), depth=depth, depth_u16=depth_u16, intr=intr,
                        backproject_float=bf, backproject_ushort=bu, thresholds=thresholds, K=K,
                        target_pc=pc, target_pix_map=pmap, **meshes)
    print("frontend_csrc:", depth.shape, [meshes[f"mesh{i}_faces"].shape[0] for i in range(4)], "faces")


def make_anchors_csrc():
    from oracle.build_ref import build
    m = build()
    cam, scene, d0, d1, pts, nodes, edges, ew = small_setup()
    rng = np.random.default_rng(17)
    bf = np.zeros((3,) + d0.shape, np.float32)
    m.backproject_depth_float(d0.astype(np.float32), bf, float(cam.fx), float(cam.fy), float(cam.cx), float(cam.cy))
    nd = np.concatenate([nodes, nodes[rng.choice(nodes.shape[0], 12, replace=False)]]).astype(np.float32)  # ties
    cov = 0.07
    pa = np.zeros((0,), np.int32)
    pw = np.zeros((0,), np.float32)
    m.compute_pixel_anchors_euclidean(nd, bf, cov, pa, pw)
    # geodesic: V vertices on pixels, quantised distances (ties), unreachable (-1) entries, invalid nodes
    V, N = 3000, 60
    H, W = 40, 90
    flat = rng.choice(H * W, V, replace=False)
    vpix = np.stack([flat % W, flat // W], 1).astype(np.int32)
    D = (np.round(rng.random((N, V)) * 40) / 100).astype(np.float32)
    D[rng.random((N, V)) < 0.3] = -1.0
    valid = (rng.random((N, 1)) > 0.15).astype(np.int32)
    verts = rng.random((V, 3)).astype(np.float32)
    ga = np.zeros((0,), np.int32)
    gw = np.zeros((0,), np.float32)
    m.compute_pixel_anchors_geodesic(D, valid, verts, vpix, ga, gw, W, H, cov)
    # update_pixel_anchors: old ids -> new ids for the valid nodes
    ids = np.nonzero(valid[:, 0])[0]
    mapping = {int(o): int(n) for n, o in enumerate(ids)}
    ra = np.where(np.isin(ga, ids), ga, -1).astype(np.int32)
    rb = ra.copy()
    m.update_pixel_anchors(mapping, rb)
    np.savez_compressed(os.path.join(HERE, "anchors_csrc.npz"), nodes=nd, point_image=bf, node_coverage=cov,
                        euclid_anchors=pa.reshape(bf.shape[1], bf.shape[2], 4),
                        euclid_weights=pw.reshape(bf.shape[1], bf.shape[2], 4),
                        geo_dist=D, geo_valid=valid, geo_vertex_pixels=vpix, geo_width=W, geo_height=H,
                        geo_anchors=ga.reshape(H, W, 4), geo_weights=gw.reshape(H, W, 4),
                        remap_in=ra, remap_ids=ids.astype(np.int32), remap_out=rb)
    print("anchors_csrc:", nd.shape[0], "nodes;", int((pa.reshape(-1, 4)[:, 0] >= 0).sum()), "anchored pixels;",
          int((ga.reshape(-1, 4)[:, 0] >= 0).sum()), "geodesic pixels")


def _graph_case(m, verts, faces, cov, K, out, tag):
    V = verts.shape[0]
    ne = m.erode_mesh(verts, faces, 1, 3)
    npos, nidx = np.zeros((0,), np.float32), np.zeros((0,), np.int32)
    n = m.sample_nodes(verts, ne, npos, nidx, cov, True, False)
    npos, nidx = npos[:n], nidx[:n]
    modes = {"valid_enforce": (True, True), "all_enforce": (False, True), "valid_prune": (True, False)}
    for name, (only_valid, enforce) in modes.items():
        E = -np.ones((n, K), np.int32)
        W = np.zeros((n, K), np.float32)
        Dd = np.zeros((n, K), np.float32)
        D = -np.ones((n, V), np.float32)
        vis = np.ones((V, 1), bool)
        m.compute_edges_geodesic(verts, vis, faces, nidx, K, cov, E, W, Dd, D, only_valid, enforce)
        out[f"{tag}_{name}_edges"], out[f"{tag}_{name}_weights"] = E, W
        out[f"{tag}_{name}_dists"], out[f"{tag}_{name}_n2v"] = Dd, D
    E = out[f"{tag}_valid_enforce_edges"]
    valid = np.ones((n, 1), bool)
    m.node_and_edge_clean_up(E, valid)
    cl = -np.ones((n, 1), np.int32)
    sizes = m.compute_clusters(E, cl)
    out.update({f"{tag}_verts": verts, f"{tag}_faces": faces, f"{tag}_cov": cov, f"{tag}_K": K,
                f"{tag}_non_eroded": ne, f"{tag}_nodes": npos, f"{tag}_node_indices": nidx,
                f"{tag}_cleanup_valid": valid, f"{tag}_clusters": cl, f"{tag}_cluster_sizes": np.array(sizes, np.int32),
                f"{tag}_euclid_edges": m.compute_edges_euclidean(npos, K)})
    print(f"graph_csrc[{tag}]:", V, "verts,", faces.shape[0], "faces,", n, "nodes,", int(valid.sum()), "kept,",
          len(sizes), "clusters")


def make_graph_csrc():
    from oracle.build_ref import build
    m = build()
    f = np.load(os.path.join(HERE, "frontend_csrc.npz"), allow_pickle=False)
    out = {}
    _graph_case(m, f["mesh0_vertices"], f["mesh0_faces"], 0.05, 8, out, "depth")
    # exact grid plane (0.01 spacing) with a hole: massive distance ties in the priority queue
    H, W = 36, 44
    yy, xx = np.mgrid[0:H, 0:W]
    P = np.stack([xx * np.float32(0.01), yy * np.float32(0.01), np.ones((H, W))]).astype(np.float32)
    P[:, 10:16, 12:20] = 0
    v = np.zeros((0,), np.float32)
    px = np.zeros((0,), np.int32)
    fc = np.zeros((0,), np.int32)
    m.compute_mesh_from_depth(P, 0.05, v, px, fc)
    _graph_case(m, v.reshape(-1, 3), fc.reshape(-1, 3), 0.045, 8, out, "grid")
    # clean-up / clusters on a sparse random graph: chains of removals, nodes invalid on entry, islands
    rng = np.random.default_rng(23)
    n, K = 300, 8
    E = -np.ones((n, K), np.int32)
    for i in range(n):
        deg = int(rng.choice([0, 1, 1, 2, 2, 3, 4, 8]))
        nb = rng.choice(np.setdiff1d(np.arange(max(0, i - 6), min(n, i + 7)), [i]), min(deg, 12), replace=False)
        E[i, :len(nb)] = nb
    valid0 = (rng.random((n, 1)) > 0.1)
    valid = valid0.copy()
    m.node_and_edge_clean_up(E, valid)
    cl = -np.ones((n, 1), np.int32)
    sizes = m.compute_clusters(E, cl)
    out.update(rand_edges=E, rand_valid_in=valid0, rand_valid_out=valid, rand_clusters=cl,
               rand_cluster_sizes=np.array(sizes, np.int32))
    print("graph_csrc[rand]:", int(valid0.sum()), "->", int(valid.sum()), "valid,", len(sizes), "clusters")
    np.savez_compressed(os.path.join(HERE, "graph_csrc.npz"), **out)


def make_integrate_small():
    cam, scene, d0, d1, pts, nodes, edges, ew = small_setup()
    origin = np.array([-0.40, -0.33, 0.95], np.float32)
    vs = 0.012
    dims = np.array([66, 52, 70])
    intr = (cam.fx, cam.fy, cam.cx, cam.cy)
    im0, im1 = S.make_image(d0), S.make_image(d1)
    world = fo.world_points(origin, dims, vs)
    V = world.shape[0]
    tsdf = np.ones(V, np.float32)
    weight = np.zeros(V, np.float32)
    color = np.zeros(V, np.float32)
    fo.integrate(tsdf, weight, color, world, np.ones(V, bool), fo.depth_of(im0), fo.pack_color(im0), intr)
    t0, w0, c0 = tsdf.copy(), weight.copy(), color.copy()
    cov = 0.07
    anchors, weights, valid = fo.skin(world, nodes, cov)
    R, T = small_transforms(scene, nodes, 1, 7)
    warped = fo.ed_warp(world, anchors, weights, valid, R, T, nodes)
    n1 = fo.integrate(tsdf, weight, color, warped, valid, fo.depth_of(im1), fo.pack_color(im1), intr)
    np.savez_compressed(os.path.join(HERE, "integrate_small.npz"), origin=origin, voxel_size=vs, dims=dims,
                        intr=np.array(intr), width=cam.width, height=cam.height, im0=im0, im1=im1, nodes=nodes,
                        node_coverage=cov, R=R, T=T, tsdf0=t0, weight0=w0, color0=c0, tsdf1=tsdf, weight1=weight,
                        color1=color, skin_valid=valid, n_updated1=n1)
    print("integrate_small:", V, "voxels,", nodes.shape[0], "nodes,", int(valid.sum()), "skinned,", n1, "updated")


def make_gn_small():
    cam, scene, d0, d1, pts, nodes, edges, ew = small_setup(seed=13)
    rng = np.random.default_rng(17)
    sel = rng.choice(pts.shape[0], 900, replace=False)
    src = pts[np.sort(sel)]
    a, w, v = fo.skin(src, nodes, 0.07)
    src, a, w = src[v][:600], a[v][:600], w[v][:600]
    tgt = (scene.deform_points(src, 2) + rng.normal(0, 0.001, src.shape)).astype(np.float32)
    tpos = scene.deform_points(nodes, 2).astype(np.float32)
    conf = np.where(rng.uniform(size=nodes.shape[0]) < 0.7, 1.0, 0.3).astype(np.float32)
    intr = np.array([cam.fx, cam.fy, cam.cx, cam.cy])
    out = fo.gn_optimize(nodes, edges, ew, tpos, conf, src, a, w, tgt, intr)
    ci = out["convergence_info"]
    np.savez_compressed(os.path.join(HERE, "gn_small.npz"), nodes=nodes, edges=edges, edge_weights=ew, tpos=tpos,
                        conf=conf, src=src, anchors=a, weights=w, tgt=tgt, intr=intr,
                        R=out["node_rotations"], t=out["node_translations"], valid=out["valid_solve"],
                        loss_total=np.array(ci["total"]))
    print("gn_small:", nodes.shape[0], "nodes,", src.shape[0], "matches, loss", ci["total"][:3], "...")


_REF = None


def _ref():
    """The reference's compiled C++ (oracle/_ref, built from /root/reference by oracle/build_ref.py)."""
    global _REF
    if _REF is None:
        from oracle.build_ref import build, load_prebuilt
        _REF = load_prebuilt() or build()
    return _REF


def csrc_depth_graph(depth, cam, coverage, max_triangle_distance=0.05, K=8):
    """SURVEY §8(d) graph of a depth frame by the REFERENCE's compiled C++, in EDGraph.from_mesh's order (the
    reference's create_graph_from_depth, embedded_deformation_graph.py:95-256): backproject_depth_float ->
    compute_mesh_from_depth -> erode_mesh(1, 3) -> sample_nodes(no shuffle, valid vertices only) ->
    compute_edges_geodesic(K, enforce) -> node_and_edge_clean_up -> the oracle's get_reduced_graph. The device
    twin is occlusionfusion_amd.synthetic.depth_graph (tests/test_gpu_golden_gn.py checks the two agree)."""
    m = _ref()
    bf = np.zeros((3,) + depth.shape, np.float32)
    m.backproject_depth_float(np.ascontiguousarray(depth, np.float32), bf, float(cam.fx), float(cam.fy),
                              float(cam.cx), float(cam.cy))
    v, px, f = np.zeros((0,), np.float32), np.zeros((0,), np.int32), np.zeros((0,), np.int32)
    m.compute_mesh_from_depth(bf, float(max_triangle_distance), v, px, f)
    v, f = v.reshape(-1, 3), f.reshape(-1, 3)
    ne = m.erode_mesh(v, f, 1, 3)
    npos, nidx = np.zeros((0,), np.float32), np.zeros((0,), np.int32)
    n = m.sample_nodes(v, ne, npos, nidx, float(coverage), True, False)
    npos, nidx = npos[:n], nidx[:n]
    E = -np.ones((n, K), np.int32)
    W = np.zeros((n, K), np.float32)
    Dd = np.zeros((n, K), np.float32)
    D = -np.ones((n, v.shape[0]), np.float32)
    m.compute_edges_geodesic(v, np.ones((v.shape[0], 1), bool), f, nidx, K, float(coverage), E, W, Dd, D, True, True)
    del D
    valid = np.ones((n, 1), bool)
    m.node_and_edge_clean_up(E, valid)
    nodes, E, W, _, _ = fo.reduced_graph(npos, E, W, Dd, -np.ones((n, 1), np.int32), valid)
    return nodes.astype(np.float32), E.astype(np.int32), W.astype(np.float32)


def config_sequence_cpu(config, rank=0):
    """BASELINE config `config`'s synthetic sequence with its SURVEY §8(d) depth-mesh graph built by the
    reference's compiled C++ (the bench builds the same graph on the device)."""
    c = S.BASELINE_CONFIGS[config]
    scene, seed = S.config_scene(config, rank)
    cam = S.bench_camera(c["cam_scale"])
    cov = S.config_coverage(config)
    g = csrc_depth_graph(S.source_depth(scene, cam, seed), cam, cov)
    return S.config_sequence(config, rank=rank, graph=g)


def config2_sequence():
    """BASELINE config 2: rigid-motion sphere + plane, 640x448, ~1k nodes (seed 2)."""
    return S.config_sequence(2)


def make_gn_1k(t=1, n_matches=10000):
    """gn_1k.npz — one DeformNet.optimize solve at a real config size (config 2: ~1k nodes, 10k matches,
    J ≈ 57k x 6k dense) by the dense f64 oracle; pins the block-sparse assembly + PCG at that size."""
    import time
    seq = config2_sequence()
    src, tgt, tpos, conf = seq.solver_inputs(t, n_matches)
    a, w, v = fo.skin(src, seq.nodes, seq.node_coverage)
    src, tgt, a, w = src[v], tgt[v], a[v], w[v]
    intr = seq.cam.as_vec()
    t0 = time.time()
    out = fo.gn_optimize(seq.nodes, seq.edges, seq.edge_weights, tpos, conf, src, a, w, tgt, intr)
    ci = out["convergence_info"]
    np.savez_compressed(os.path.join(HERE, "gn_1k.npz"), nodes=seq.nodes, edges=seq.edges,
                        edge_weights=seq.edge_weights, node_coverage=seq.node_coverage, tpos=tpos, conf=conf,
                        src=src, anchors=a, weights=w, tgt=tgt, intr=intr, frame=t,
                        R=out["node_rotations"], t=out["node_translations"], valid=out["valid_solve"],
                        loss_total=np.array(ci["total"]))
    print("gn_1k:", seq.nodes.shape[0], "nodes,", src.shape[0], "matches, loss", ci["total"][:3], "...",
          f"{time.time() - t0:.0f} s")


def _frame_problem(seq, t, n_matches=10000):
    """Frame t's GN inputs exactly as FusionPipeline.prepare builds them: seeded matches + node targets, then the
    skin of the source points (oracle skin == the device skin, tests/test_gpu_parity.py) keeping the valid ones."""
    src, tgt, tpos, conf = seq.solver_inputs(t, n_matches)
    a, w, v = fo.skin(src, seq.nodes, seq.node_coverage)
    return dict(src=src[v], tgt=tgt[v], tpos=tpos, conf=conf, anchors=a[v], weights=w[v])


def make_gn_chain(name, config, frames, n_matches=10000, rank=0):
    """gn_2k.npz / gn_4k.npz — DeformNet.optimize (model.py:222-859) at the headline sizes by the f64 oracle
    (gn_optimize_sparse: the dense restatement's rows with a sparse JᵀJ, then the reference's dense LU), on
    BASELINE config `config`'s occluded non-rigid frames with its SURVEY §8(d) depth-mesh graph (the reference's
    compiled C++). frames = (t0, t1, ...): t0 starts from the identity, every later frame from the previous
    frame's oracle result (the frame loop's prev_rot / prev_trans). Config 5: `rank`'s independent scene
    (synthetic.config_scene)."""
    import time
    seq = config_sequence_cpu(config, rank)
    intr = seq.cam.as_vec()
    out = dict(nodes=seq.nodes, edges=seq.edges, edge_weights=seq.edge_weights, node_coverage=seq.node_coverage,
               intr=intr, config=config, frames=np.array(frames, np.int32), seed=seq.seed, rank=rank)
    R = T = None
    for q, t in enumerate(frames):
        pb = _frame_problem(seq, t, n_matches)
        t0 = time.time()
        res = fo.gn_optimize_sparse(seq.nodes, seq.edges, seq.edge_weights, pb["tpos"], pb["conf"], pb["src"],
                                    pb["anchors"], pb["weights"], pb["tgt"], intr, prev_rot=R, prev_trans=T)
        R, T = res["node_rotations"], res["node_translations"]
        ci = res["convergence_info"]
        for k, v in pb.items():
            out[f"f{q}_{k}"] = v
        out.update({f"f{q}_R": R, f"f{q}_t": T, f"f{q}_valid": res["valid_solve"],
                    f"f{q}_loss_total": np.array(ci["total"]), f"f{q}_loss_data": np.array(ci["data"])})
        print(f"{name} frame {t}: {seq.nodes.shape[0]} nodes, {pb['src'].shape[0]} matches, "
              f"{int((pb['conf'] < 1).sum())} low-confidence nodes, {len(ci['total'])} GN steps, loss "
              f"{ci['total'][0]:.6f} -> {ci['total'][-1]:.6f} ({time.time() - t0:.0f} s)", flush=True)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)


HOLE_CENTER = (0.10, -0.05, 1.10)   # a point on the sphere's visible front (config 3's scene)
HOLE_RADIUS = 0.12


def make_gn_hole():
    """gn_2k_hole.npz — a differently conditioned spectrum at the headline size (round 6): gn_2k's frame 10 with every
    match anchored to a node within 12 cm of a point on the sphere's front removed, and those nodes' motion-term
    confidence set to 0.3, so a 48-node patch is held only by ARAP and confidence-0.3 motion rows; solved by the
    f64 oracle (gn_optimize_sparse) from the identity."""
    import time
    g = np.load(os.path.join(HERE, "gn_2k.npz"), allow_pickle=False)
    nodes = g["nodes"]
    c = nodes[np.argmin(((nodes - np.asarray(HOLE_CENTER, np.float32)) ** 2).sum(1))]
    hole = np.sqrt(((nodes - c) ** 2).sum(1)) < HOLE_RADIUS
    keep = ~hole[g["f0_anchors"]].any(1)
    conf = g["f0_conf"].copy()
    conf[hole] = np.float32(0.3)
    pb = dict(src=g["f0_src"][keep], tgt=g["f0_tgt"][keep], tpos=g["f0_tpos"], conf=conf,
              anchors=g["f0_anchors"][keep], weights=g["f0_weights"][keep])
    intr = g["intr"]
    t0 = time.time()
    res = fo.gn_optimize_sparse(nodes, g["edges"], g["edge_weights"], pb["tpos"], pb["conf"], pb["src"], pb["anchors"],
                                pb["weights"], pb["tgt"], intr)
    ci = res["convergence_info"]
    out = dict(nodes=nodes, edges=g["edges"], edge_weights=g["edge_weights"], node_coverage=g["node_coverage"],
               intr=intr, config=g["config"], frames=np.array([10], np.int32), seed=g["seed"], hole=hole)
    out.update({f"f0_{k}": v for k, v in pb.items()})
    out.update(f0_R=res["node_rotations"], f0_t=res["node_translations"], f0_valid=res["valid_solve"],
               f0_loss_total=np.array(ci["total"]), f0_loss_data=np.array(ci["data"]))
    np.savez_compressed(os.path.join(HERE, "gn_2k_hole.npz"), **out)
    print(f"gn_2k_hole: {int(hole.sum())} hole nodes, {pb['src'].shape[0]} matches, {len(ci['total'])} GN steps, loss "
          f"{ci['total'][0]:.6f} -> {ci['total'][-1]:.6f} ({time.time() - t0:.0f} s)", flush=True)


MOOSE = "/root/reference/NonRigidICP/demo/moose6OK9_AttackTrotRM"   # read here only; the fixture travels


def moose_inputs():
    """The reference's real demo pair (NonRigidICP/config.yaml: src = depth/cam1_0015.png, tgt = cam1_0009.png,
    cam1intr.txt, Lepard landmarks landmark/moose_match_pred.npz; loaded as NonRigidICP/main.py:35-48 does).
    -> (src_mm, tgt_mm uint16 (500, 512), K 3x3, uv_src, uv_tgt (455, 2) int64)."""
    from PIL import Image
    src_mm = np.array(Image.open(os.path.join(MOOSE, "depth/cam1_0015.png")))
    tgt_mm = np.array(Image.open(os.path.join(MOOSE, "depth/cam1_0009.png")))
    assert src_mm.dtype == np.uint16 and tgt_mm.dtype == np.uint16
    K = np.loadtxt(os.path.join(MOOSE, "cam1intr.txt"))
    lm = np.load(os.path.join(MOOSE, "landmark/moose_match_pred.npz"), allow_pickle=False)
    ldmk_src = lm["src_pcd"][0][lm["match"][:, 1]]
    ldmk_tgt = lm["tgt_pcd"][0][lm["match"][:, 2]]
    return src_mm, tgt_mm, K, fo.xyz_2_uv(ldmk_src, K), fo.xyz_2_uv(ldmk_tgt, K)


MOOSE_COVERAGE = 0.09          # NonRigidICP/model/geometry.py:123 (node_coverage, metres)
MOOSE_MAX_TRIANGLE = 0.04      # geometry.py:117


def moose_problem(src_mm, tgt_mm, K, uv_src, uv_tgt, nodes):
    """The landmark GN problem on the §8 path's conventions: depth in metres as f32(mm) / f32(1000)
    (backproject_depth's ushort branch), both clouds by depth_2_pc + map_pixel_to_pcd (registration_fusion.py:
    104-109, 388-395: f64 from the f32 depth, then f32), landmark pixels looked up as registration.py:76-84 does
    (pairs whose source or target pixel has no depth dropped), skinned by WarpField.skin (k-NN, node coverage)
    keeping the valid ones. -> dict(src, tgt, anchors, weights, keep)."""
    f32 = np.float32
    ds, dt = src_mm.astype(f32) / f32(1000.0), tgt_mm.astype(f32) / f32(1000.0)
    spc, smap = fo.target_point_cloud(ds, K)
    tpc, tmap = fo.target_point_cloud(dt, K)
    H, W = ds.shape
    inb = ((uv_src[:, 0] >= 0) & (uv_src[:, 0] < W) & (uv_src[:, 1] >= 0) & (uv_src[:, 1] < H)
           & (uv_tgt[:, 0] >= 0) & (uv_tgt[:, 0] < W) & (uv_tgt[:, 1] >= 0) & (uv_tgt[:, 1] < H))
    assert inb.all()
    s_id = smap[uv_src[:, 1], uv_src[:, 0]]
    t_id = tmap[uv_tgt[:, 1], uv_tgt[:, 0]]
    ok = (s_id > -1) & (t_id > -1)
    src, tgt = spc[s_id[ok]], tpc[t_id[ok]]
    a, w, v = fo.skin(src, nodes, MOOSE_COVERAGE)
    keep = np.nonzero(ok)[0][v]
    return dict(src=src[v], tgt=tgt[v], anchors=a[v], weights=w[v], keep=keep.astype(np.int32))


def make_moose():
    """moose.npz — the reference's real inputs through the hot path: the depth pair + intrinsics + the landmark
    pixels (inputs), the SURVEY §8(d) depth-mesh graph of the source frame by the reference's compiled C++ with the
    demo's coverage / triangle size, the landmark GN problem (moose_problem) and its DeformNet.optimize solve by
    the dense f64 oracle (data rows: λ_depth = 1, λ_flow = 0 — 3-D landmark residuals, as landmark_cost; ARAP;
    no node-motion targets), and a 128³ volume around the source cloud for the warped integrate. Parity of these
    outputs against the reference itself is unpinned (its Python cannot run here)."""
    src_mm, tgt_mm, K, uv_src, uv_tgt = moose_inputs()
    cam = S.Intrinsics(float(K[0, 0]), float(K[1, 1]), float(K[0, 2]), float(K[1, 2]), src_mm.shape[1],
                       src_mm.shape[0])
    depth_m = src_mm.astype(np.float32) / np.float32(1000.0)
    nodes, edges, ew = csrc_depth_graph(depth_m, cam, MOOSE_COVERAGE, max_triangle_distance=MOOSE_MAX_TRIANGLE)
    pb = moose_problem(src_mm, tgt_mm, K, uv_src, uv_tgt, nodes)
    N = nodes.shape[0]
    intr = cam.as_vec()
    res = fo.gn_optimize(nodes, edges, ew, nodes.copy(), np.zeros(N, np.float32), pb["src"], pb["anchors"],
                         pb["weights"], pb["tgt"], intr)
    ci = res["convergence_info"]
    spc, _ = fo.target_point_cloud(depth_m, K)
    lo, hi = spc.min(0), spc.max(0)
    vs = np.float32(np.ceil((hi - lo).max() * 1.2 / 128 * 1000) / 1000)       # whole mm
    origin = ((lo + hi) / 2 - vs * 64).astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "moose.npz"), src_mm=src_mm, tgt_mm=tgt_mm, K=K, uv_src=uv_src,
                        uv_tgt=uv_tgt, nodes=nodes, edges=edges, edge_weights=ew, node_coverage=MOOSE_COVERAGE,
                        max_triangle_distance=MOOSE_MAX_TRIANGLE, **pb, R=res["node_rotations"],
                        t=res["node_translations"], valid=res["valid_solve"], loss_total=np.array(ci["total"]),
                        origin=origin, voxel_size=vs, dims=np.array([128, 128, 128]))
    print(f"moose: {N} nodes, {pb['src'].shape[0]} of {uv_src.shape[0]} landmarks, loss {ci['total'][0]:.6g} -> "
          f"{ci['total'][-1]:.6g} in {len(ci['total'])} steps, volume origin {origin} voxel {vs}")


if __name__ == "__main__":
    which = sys.argv[1:] or ["skin", "frontend", "anchors", "graph", "integrate", "gn", "gn1k", "gn2k", "gn4k",
                             "moose"]
    if "moose" in which:
        make_moose()
    if "gn2k" in which:
        make_gn_chain("gn_2k", 3, (10, 11))
    if "gn4k" in which:
        make_gn_chain("gn_4k", 4, (10,))
    if "hole" in which:
        make_gn_hole()
    if "gn5" in which:   # BASELINE config 5: rank 1's and rank 7's independent scenes (one GPU each)
        make_gn_chain("gn_c5r1", 5, (10,), rank=1)
        make_gn_chain("gn_c5r7", 5, (10,), rank=7)
    if "gn1k" in which:
        make_gn_1k()
    if "skin" in which:
        make_skin_csrc()
    if "frontend" in which:
        make_frontend_csrc()
    if "anchors" in which:
        make_anchors_csrc()
    if "graph" in which:
        make_graph_csrc()
    if "integrate" in which:
        make_integrate_small()
    if "gn" in which:
        make_gn_small()
