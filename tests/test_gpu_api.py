"""GPU: the reference API conventions around the hot path.

* a9 — WarpField.update_transformations / get_transformation_wrt_graph_node / get_transformation_wrt_origin
  (fusion_with_occlusion/warpfield.py:389-449): the warp field keeps the solver's node-relative (R, T), its
  `translations` are the origin form t = -R g + g + T restated with the reference's own per-node loop, the two
  conversions invert each other, deformed nodes / frame id are taken over, a frame mismatch asserts, and the
  origin-form LBS warp (deform_lbs) equals the node-relative ED warp (deform_ED) of the same transforms.
* a12 — Registration.optimize (NonRigidICP/model/registration_fusion.py:98-145, returns :363-377): the dict's
  keys, types and dtypes (rotations numpy f64 from scipy's as_matrix, translations a CPU tensor, deformed nodes
  and warped vertices device tensors, frame ids from optical_flow_data), the target cloud / pixel map, and the
  solve itself — within 1e-5 of the dense f64 oracle (model.py:222-859) on exactly the matches the API selects.
"""
import os

import numpy as np
import pytest
import torch

from oracle import fusion_oracle as fo

pytestmark = pytest.mark.gpu


class _Opt:
    source_frame = 0
    skip_rate = 1


@pytest.fixture(scope="module")
def setup(cuda, golden_dir):
    from occlusionfusion_amd import EDGraph, TSDFVolume, WarpField
    from occlusionfusion_amd.synthetic import euclidean_edges
    g = np.load(os.path.join(golden_dir, "integrate_small.npz"), allow_pickle=False)
    vol = TSDFVolume.from_grid(g["origin"], float(g["voxel_size"]), g["dims"], tuple(g["intr"]), _Opt(), device=cuda)
    vol.integrate({"im": g["im0"], "id": 0})
    e, w = euclidean_edges(g["nodes"], 8)
    graph = EDGraph(g["nodes"], e, w, node_coverage=float(g["node_coverage"]))
    return g, vol, graph, WarpField(graph, vol)


def _ref_origin_form(R, T, nodes):
    """warpfield.py:407-408 verbatim in numpy: -[R_i @ g_i] + g + T."""
    N = nodes.shape[0]
    return -np.array([R[i] @ nodes[i] for i in range(N)]) + nodes + T


def test_a9_update_transformations_and_conventions(setup):
    g, vol, graph, wf = setup
    N = graph.nodes.shape[0]
    rng = np.random.default_rng(3)
    R = fo.angle_axis_to_rotation_matrix(rng.normal(0, 0.05, (N, 3))).astype(np.float32)
    T = rng.normal(0, 0.01, (N, 3)).astype(np.float32)
    wf.frame_id = vol.frame_id
    dn = (graph.nodes + T).astype(np.float32)
    wf.update_transformations({"node_rotations": R, "node_translations": T, "deformed_nodes_to_target": dn,
                               "target_frame_id": 1})
    assert wf.frame_id == 1
    np.testing.assert_array_equal(wf.deformed_nodes, dn)
    np.testing.assert_array_equal(wf.rotations, R)
    t_origin = wf.translations
    np.testing.assert_allclose(t_origin, _ref_origin_form(R, T, graph.nodes), atol=1e-6)
    np.testing.assert_allclose(t_origin, fo.to_origin_form(R.astype(np.float64), T, graph.nodes), atol=1e-6)
    R2, T2 = wf.get_transformation_wrt_graph_node()
    np.testing.assert_array_equal(R2, R)
    np.testing.assert_allclose(T2, T, atol=1e-6)
    R3, t3 = wf.get_transformation_wrt_origin(R2, T2)          # warpfield.py:438-449
    np.testing.assert_allclose(t3, t_origin, atol=1e-6)
    # origin-form LBS (warpfield.py:208-231) == node-relative ED warp (geometry.py:9-25) of the same transforms
    pts = (g["nodes"][rng.integers(0, N, 2000)] + rng.normal(0, 0.02, (2000, 3))).astype(np.float32)
    a, w, v = wf.skin(pts)
    ed = wf.deform_device(pts, a, w, v).cpu().numpy()
    lbs = wf.deform_lbs(R, t_origin.astype(np.float32), pts, a, w, v)
    np.testing.assert_allclose(lbs, ed, atol=2e-6)
    # tsdf.frame_id is still 0: a second update must refuse (warpfield.py:399)
    with pytest.raises(AssertionError):
        wf.update_transformations({"node_rotations": R, "node_translations": T, "deformed_nodes_to_target": dn,
                                   "target_frame_id": 2})
    wf.frame_id = vol.frame_id


def test_a12_registration_optimize_dict_contract(setup, cuda):
    from occlusionfusion_amd import synthetic as S
    from occlusionfusion_amd.registration import Registration
    g, vol, graph, wf = setup
    cam = S.Intrinsics(*(float(x) for x in g["intr"]), int(g["width"]), int(g["height"]))
    rng = np.random.default_rng(11)
    verts = S.backproject(g["im0"][5], cam)
    verts = verts[rng.permutation(verts.shape[0])[:4000]]
    K = np.eye(3)
    K[0, 0], K[1, 1], K[0, 2], K[1, 2] = g["intr"]
    wf.set_node_transforms(np.tile(np.eye(3, dtype=np.float32), (graph.nodes.shape[0], 1, 1)),
                           np.zeros((graph.nodes.shape[0], 3), np.float32))
    reg = Registration(verts, graph, wf, K)
    scene = S.SphereScene()
    matches = (scene.deform_points(verts, 1) + rng.normal(0, 0.001, verts.shape)).astype(np.float32)
    valid_verts = rng.random(verts.shape[0]) < 0.9
    N = graph.nodes.shape[0]
    tpos = scene.deform_points(graph.nodes, 1).astype(np.float32)
    conf = np.where(rng.random(N) < 0.8, 1.0, 0.3).astype(np.float32)
    out = reg.optimize({"source_id": 0, "target_id": 1}, {"target_matches": matches, "valid_verts": valid_verts},
                       (tpos, conf), {"im": g["im1"]})
    for k in ("warped_verts", "node_rotations", "node_translations", "deformed_nodes_to_target", "convergence_info",
              "source_frame_id", "target_frame_id"):
        assert k in out, k
    assert out["source_frame_id"] == 0 and out["target_frame_id"] == 1
    Rr, Tt = out["node_rotations"], out["node_translations"]
    assert isinstance(Rr, np.ndarray) and Rr.dtype == np.float64 and Rr.shape == (N, 3, 3)
    assert isinstance(Tt, torch.Tensor) and Tt.device.type == "cpu" and Tt.dtype == torch.float32 and Tt.shape == (N, 3)
    dn = out["deformed_nodes_to_target"]
    assert isinstance(dn, torch.Tensor) and dn.device.type == "cuda"
    np.testing.assert_array_equal(dn.cpu().numpy(), graph.nodes + Tt.numpy())
    assert isinstance(out["convergence_info"], dict) and len(out["convergence_info"]["total"]) >= 1
    # target cloud of the target frame (registration_fusion.py:104-109)
    d1 = g["im1"][5]
    assert reg.tgt_pcd.shape == (int((d1 > 0).sum()), 3)
    # the solve on exactly the matches the API selects, against the dense oracle
    a, w, v = fo.skin(verts, graph.nodes, wf.node_coverage)
    src, an, wt = verts[v], a[v], w[v]
    sel = np.nonzero(valid_verts[: src.shape[0]])[0]
    ref = fo.gn_optimize(graph.nodes, graph.edges, graph.edges_weights, tpos, conf, src[sel], an[sel], wt[sel],
                         matches[v][sel], g["intr"])
    assert ref["valid_solve"] == 1
    assert np.abs(Rr - ref["node_rotations"]).max() < 1e-5
    assert np.abs(Tt.numpy() - ref["node_translations"]).max() < 1e-5
    # warped_verts = deform_ED of the valid source vertices with the result (geometry.py:9-25), bit-exact
    wv = out["warped_verts"]
    assert wv.device.type == "cuda" and wv.shape == (src.shape[0], 3)
    exp = fo.ed_warp(src, an, wt, np.ones(src.shape[0], bool), Rr.astype(np.float32), Tt.numpy(), graph.nodes)
    np.testing.assert_array_equal(wv.cpu().numpy(), exp)
