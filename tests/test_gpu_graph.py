"""GPU parity of ED-graph construction through the C ABI: erode_mesh, sample_nodes,
compute_edges_geodesic (three modes), compute_edges_euclidean, node_and_edge_clean_up, compute_clusters
(csrc/cpu/graph_proc.cpp:17-481) and EDGraph.from_mesh (embedded_deformation_graph.py:174-380).

Pinned by tests/golden/graph_csrc.npz, the outputs of the REFERENCE's compiled C++: bit-exact (edge
weights within 4 ulp: glibc expf), including the priority-queue tie order on an exact grid mesh."""
import os

import numpy as np
import pytest
import torch

from oracle import fusion_oracle as fo

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def g(golden_dir):
    return np.load(os.path.join(golden_dir, "graph_csrc.npz"), allow_pickle=False)


def _ulps(a, b):
    return int(np.abs(a.view(np.int32).astype(np.int64) - b.view(np.int32).astype(np.int64)).max(initial=0))


@pytest.mark.parametrize("tag", ["depth", "grid"])
def test_graph_construction_matches_csrc(g, cuda, tag):
    from occlusionfusion_amd.graph_proc import (MeshGraph, clusters_device, edges_euclidean_device,
                                                node_edge_cleanup_device)
    V, F = g[f"{tag}_verts"], g[f"{tag}_faces"]
    cov, K = float(g[f"{tag}_cov"]), int(g[f"{tag}_K"])
    mg = MeshGraph(V, F, cuda)
    rp, col = mg.adjacency()
    nb = fo.vertex_neighbors(F, V.shape[0])
    assert np.array_equal(rp.cpu().numpy(), np.concatenate([[0], np.cumsum([len(x) for x in nb])]))
    assert np.array_equal(col.cpu().numpy(), np.concatenate([np.array(x, np.int64) for x in nb]).astype(np.int32))
    ne = mg.erode(1, 3)
    assert np.array_equal(ne.cpu().numpy(), g[f"{tag}_non_eroded"].reshape(-1))
    pos, idx = mg.sample_nodes(ne, cov)
    assert np.array_equal(pos.cpu().numpy(), g[f"{tag}_nodes"])
    assert np.array_equal(idx.cpu().numpy(), g[f"{tag}_node_indices"].reshape(-1))
    for name, (ov, en) in {"valid_enforce": (True, True), "all_enforce": (False, True),
                           "valid_prune": (True, False)}.items():
        E, W, D, n2v = mg.edges_geodesic(idx, K, cov, ov, en, with_node_to_vertex=True)
        assert np.array_equal(E.cpu().numpy(), g[f"{tag}_{name}_edges"]), name
        assert np.array_equal(D.cpu().numpy(), g[f"{tag}_{name}_dists"]), name
        assert np.array_equal(n2v.cpu().numpy(), g[f"{tag}_{name}_n2v"]), name
        assert _ulps(W.cpu().numpy(), g[f"{tag}_{name}_weights"]) <= 4, name
    assert np.array_equal(edges_euclidean_device(pos, K).cpu().numpy(), g[f"{tag}_euclid_edges"])
    E = torch.from_numpy(g[f"{tag}_valid_enforce_edges"]).to(cuda)
    valid = node_edge_cleanup_device(E, torch.ones(E.shape[0], dtype=torch.bool, device=cuda))
    assert np.array_equal(valid.cpu().numpy(), g[f"{tag}_cleanup_valid"].reshape(-1))
    cl, sizes = clusters_device(E)
    assert np.array_equal(cl.cpu().numpy(), g[f"{tag}_clusters"].reshape(-1))
    assert sizes == list(g[f"{tag}_cluster_sizes"])


def test_cleanup_and_clusters_random_graph(g, cuda):
    from occlusionfusion_amd.graph_proc import compute_clusters, node_and_edge_clean_up
    valid = g["rand_valid_in"].copy()
    node_and_edge_clean_up(g["rand_edges"], valid)
    assert np.array_equal(valid, g["rand_valid_out"])
    cl = -np.ones((g["rand_edges"].shape[0], 1), np.int32)
    assert compute_clusters(g["rand_edges"], cl) == list(g["rand_cluster_sizes"])
    assert np.array_equal(cl, g["rand_clusters"])


def test_csrc_call_shapes(g, cuda):
    from occlusionfusion_amd import graph_proc as gp
    V, F = g["grid_verts"], g["grid_faces"]
    ne = gp.erode_mesh(V, F, 1, 3)
    assert ne.shape == (V.shape[0], 1) and np.array_equal(ne, g["grid_non_eroded"])
    npos, nidx = np.zeros((0,), np.float32), np.zeros((0,), np.int32)
    n = gp.sample_nodes(V, ne, npos, nidx, float(g["grid_cov"]), True, False)
    assert npos.shape == (V.shape[0], 3) and np.array_equal(npos[:n], g["grid_nodes"])
    assert np.array_equal(nidx[:n], g["grid_node_indices"])
    K = int(g["grid_K"])
    E, W = -np.ones((n, K), np.int32), np.zeros((n, K), np.float32)
    D, N2V = np.zeros((n, K), np.float32), -np.ones((n, V.shape[0]), np.float32)
    gp.compute_edges_geodesic(V, np.ones((V.shape[0], 1), bool), F, nidx[:n], K, float(g["grid_cov"]), E, W, D, N2V,
                              True, True)
    assert np.array_equal(E, g["grid_valid_enforce_edges"]) and np.array_equal(N2V, g["grid_valid_enforce_n2v"])
    # random shuffle: a valid sampling (every eligible vertex covered, nodes pairwise > coverage apart)
    n2 = gp.sample_nodes(V, ne, npos, nidx, float(g["grid_cov"]), True, True)
    P = npos[:n2]
    d2 = fo._eigen_sqnorm(P[:, None, :] - P[None, :, :])
    c2 = np.float32(g["grid_cov"]) * np.float32(g["grid_cov"])
    assert (d2[~np.eye(n2, dtype=bool)] > c2).all()


def test_sample_nodes_and_geodesic_large_mesh(cuda):
    """A 512x512 grid-like noisy depth mesh (~250k vertices): sample_nodes equals the oracle's sequential
    sampling; geodesic edges are deterministic and well formed (the Python Dijkstra is too slow here)."""
    from occlusionfusion_amd.graph_proc import MeshGraph
    from occlusionfusion_amd.image_proc import compute_mesh_from_depth_device
    rng = np.random.default_rng(4)
    H, W = 512, 512
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float32)
    z = (1.2 + 0.1 * np.sin(xx / 40) * np.cos(yy / 55) + rng.normal(0, 0.0005, (H, W))).astype(np.float32)
    P = np.stack([(xx - 256) * z / 500, (yy - 256) * z / 500, z]).astype(np.float32)
    m = compute_mesh_from_depth_device(torch.from_numpy(P).to(cuda), 0.05)
    mg = MeshGraph(m["vertices"], m["faces"], cuda)
    ne = mg.erode(1, 3)
    pos, idx = mg.sample_nodes(ne, 0.05)
    vn = m["vertices"].cpu().numpy()
    opos, oidx = fo.sample_nodes(vn, ne.cpu().numpy(), 0.05)
    assert np.array_equal(idx.cpu().numpy(), oidx.reshape(-1)) and np.array_equal(pos.cpu().numpy(), opos)
    E1, W1, D1, _ = mg.edges_geodesic(idx, 8, 0.05)
    E2, W2, D2, _ = mg.edges_geodesic(idx, 8, 0.05)
    assert torch.equal(E1, E2) and torch.equal(W1, W2) and torch.equal(D1, D2)
    E = E1.cpu().numpy()
    assert (E >= 0).all() and (E < idx.shape[0]).all()
    assert (E != np.arange(E.shape[0])[:, None]).all()
    assert np.allclose(W1.sum(1).cpu().numpy(), 1, atol=1e-5)
    assert (np.diff(D1.cpu().numpy(), axis=1) >= 0).all()     # neighbours in non-decreasing geodesic distance
