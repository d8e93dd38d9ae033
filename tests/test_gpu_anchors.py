"""GPU parity of the standalone skinning / anchor ops through the C ABI:
csrc compute_pixel_anchors_euclidean / _geodesic and update_pixel_anchors (graph_proc.cpp:483-709,934-961),
the k-NN query behind WarpField.find_unreachable_nodes (warpfield.py:462-485) and WarpField.skin_image
(warpfield.py:143-199).

Pinned by tests/golden/anchors_csrc.npz (outputs of the REFERENCE's compiled C++): anchors bit-exact
(including the tie order of duplicated nodes and the std::set distance dedupe), weights within 4 ulp (glibc
expf vs the correctly rounded exp) and bit-exact against the oracle restatement."""
import os

import numpy as np
import pytest
import torch

from oracle import fusion_oracle as fo

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def g(golden_dir):
    return np.load(os.path.join(golden_dir, "anchors_csrc.npz"), allow_pickle=False)


def _ulps(a, b):
    return int(np.abs(a.view(np.int32).astype(np.int64) - b.view(np.int32).astype(np.int64)).max(initial=0))


def test_pixel_anchors_euclidean(g, cuda):
    from occlusionfusion_amd.graph_proc import compute_pixel_anchors_euclidean
    a, w = np.zeros((0,), np.int32), np.zeros((0,), np.float32)
    compute_pixel_anchors_euclidean(g["nodes"], g["point_image"], float(g["node_coverage"]), a, w)
    assert np.array_equal(a, g["euclid_anchors"])
    assert _ulps(w, g["euclid_weights"]) <= 4
    oa, ow = fo.pixel_anchors_euclidean(g["nodes"], g["point_image"], float(g["node_coverage"]))
    assert np.array_equal(a, oa) and np.array_equal(w, ow)


def test_pixel_anchors_geodesic(g, cuda):
    from occlusionfusion_amd.graph_proc import compute_pixel_anchors_geodesic
    a, w = np.zeros((0,), np.int32), np.zeros((0,), np.float32)
    W, H = int(g["geo_width"]), int(g["geo_height"])
    verts = np.zeros((g["geo_vertex_pixels"].shape[0], 3), np.float32)
    compute_pixel_anchors_geodesic(g["geo_dist"], g["geo_valid"], verts, g["geo_vertex_pixels"], a, w, W, H,
                                   float(g["node_coverage"]))
    assert np.array_equal(a, g["geo_anchors"])
    assert _ulps(w, g["geo_weights"]) <= 4
    oa, ow = fo.pixel_anchors_geodesic(g["geo_dist"], g["geo_valid"], g["geo_vertex_pixels"], W, H,
                                       float(g["node_coverage"]))
    assert np.array_equal(a, oa) and np.array_equal(w, ow)


def test_update_pixel_anchors(g, cuda):
    from occlusionfusion_amd.graph_proc import update_pixel_anchors
    mapping = {int(o): n for n, o in enumerate(g["remap_ids"])}
    a = g["remap_in"].copy()
    update_pixel_anchors(mapping, a)
    assert np.array_equal(a, g["remap_out"])
    bad = g["remap_in"].copy()
    invalid = np.setdiff1d(np.arange(g["geo_valid"].shape[0]), g["remap_ids"])
    bad.reshape(-1)[np.nonzero(bad.reshape(-1) >= 0)[0][0]] = invalid[0]   # no mapping -> map::at throws
    with pytest.raises(IndexError):
        update_pixel_anchors(mapping, bad)


@pytest.mark.parametrize("k", [1, 4, 8])
def test_knn_matches_oracle(cuda, k):
    from occlusionfusion_amd.graph_proc import knn_device
    rng = np.random.default_rng(k)
    nodes = rng.random((2100, 3)).astype(np.float32)
    nodes[7] = nodes[3]                      # a tie: equal distance, lower id first
    pts = rng.random((20000, 3)).astype(np.float32)
    pts[0] = nodes[3]
    idx, d2 = knn_device(torch.from_numpy(pts).to(cuda), torch.from_numpy(nodes).to(cuda), k)
    oi, od = fo.knn(pts, nodes, k)
    assert np.array_equal(idx.cpu().numpy(), oi) and np.array_equal(d2.cpu().numpy(), od)
    if k > 1:
        assert idx[0, :2].cpu().tolist() == [3, 7]
    idx, d2 = knn_device(torch.from_numpy(pts[:50]).to(cuda), torch.from_numpy(nodes[:3]).to(cuda), 8)
    assert (idx[:, 3:] == -1).all() and torch.isinf(d2[:, 3:]).all()


def _warpfield(nodes, cov=0.07):
    from types import SimpleNamespace
    from occlusionfusion_amd import EDGraph, TSDFVolume, WarpField
    from occlusionfusion_amd.synthetic import euclidean_edges
    vol = TSDFVolume.from_grid(np.array([-0.4, -0.3, 1.0], np.float32), 0.02, (16, 16, 16), (100., 100., 8., 8.),
                               SimpleNamespace(source_frame=0, skip_rate=1))
    e, w = euclidean_edges(nodes, 8)
    return WarpField(EDGraph(nodes, e, w, node_coverage=cov), vol)


def test_find_unreachable_nodes(g, cuda):
    nodes = g["nodes"][:200]
    wf = _warpfield(nodes)
    rng = np.random.default_rng(2)
    pts = (nodes[rng.integers(0, 200, 5000)] + rng.normal(0, 0.12, (5000, 3))).astype(np.float32)
    got = wf.find_unreachable_nodes(pts)
    exp = fo.find_unreachable_nodes(pts, nodes, wf.node_coverage)
    assert len(got) > 100 and np.array_equal(np.asarray(got), np.asarray(exp))
    assert wf.find_unreachable_nodes(nodes[:10]) == []


def test_skin_image(g, cuda, golden_dir):
    f = np.load(os.path.join(golden_dir, "frontend_csrc.npz"), allow_pickle=False)
    P = f["backproject_float"]
    nodes = g["nodes"][:200]
    wf = _warpfield(nodes)
    im = np.concatenate([np.zeros_like(P), P])
    mask = np.ones(P.shape[1:], np.float32)
    mask[:, :40] = 0
    out = wf.skin_image(nodes, {"im": im, "mask": mask})
    # oracle: mesh of the masked point image -> skin of its vertices -> scatter (zeros elsewhere)
    v, px, _ = fo.compute_mesh_from_depth(P * mask[None], 0.05)
    a, w, _ = fo.skin(v, nodes, wf.node_coverage)
    ea = np.zeros(P.shape[1:] + (4,), np.int32)
    ew = np.zeros(P.shape[1:] + (4,), np.float32)
    ea[px[:, 1], px[:, 0]] = a
    ew[px[:, 1], px[:, 0]] = w
    assert np.array_equal(out["pixel_anchors"], ea) and np.array_equal(out["pixel_weights"], ew)
    assert (out["pixel_anchors"][:, :40] == 0).all() and (out["pixel_anchors"] > 0).any()
