"""Device twins of the reference's C++ graph utilities (NeuralNRT._C, csrc/cpu/graph_proc.cpp) with the
pybind call shapes its Python callers use (outputs are arrays resized in place). SURVEY §8(f) rows 2 and 4.

  compute_pixel_anchors_euclidean   graph_proc.cpp:610-709  -> ofx_pixel_anchors_euclidean
  compute_pixel_anchors_geodesic    graph_proc.cpp:483-608  -> ofx_pixel_anchors_geodesic
  update_pixel_anchors              graph_proc.cpp:934-961  -> ofx_remap_anchors
  knn (pykdtree KDTree.query)       warpfield.py:103-104     -> ofx_knn_points

Bit-exact with the compiled reference except the last bits of skinning weights (glibc expf vs the correctly
rounded exp; tests/test_gpu_anchors.py). There is no CPU fallback.
"""
import numpy as np
import torch

from . import _lib
from ._lib import call, ptr, stream_ptr

GRAPH_K = 4   # csrc/cpu/graph_proc.h:8


def _dev(device):
    return torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())


def _t(x, device, dtype):
    if isinstance(x, torch.Tensor):
        return x.to(device=device, dtype=dtype).contiguous()
    return torch.as_tensor(np.ascontiguousarray(x), device=device).to(dtype).contiguous()


def _fill_inplace(arr, t):
    arr.resize(tuple(t.shape), refcheck=False)
    arr[...] = t.cpu().numpy()


def pixel_anchors_euclidean_device(nodes, point_image, node_coverage):
    """(nodes (N,3), point image (3,H,W)) device tensors -> (anchors (H,W,4) i32, weights (H,W,4) f32)."""
    P = point_image.contiguous().float()
    _, H, W = P.shape
    nd = nodes.contiguous().float().reshape(-1, 3)
    a = torch.empty((H, W, GRAPH_K), dtype=torch.int32, device=P.device)
    w = torch.empty((H, W, GRAPH_K), dtype=torch.float32, device=P.device)
    call("ofx_pixel_anchors_euclidean", ptr(nd), nd.shape[0], ptr(P), H, W, float(node_coverage), ptr(a), ptr(w),
         stream_ptr())
    return a, w


def compute_pixel_anchors_euclidean(graph_nodes, point_image, node_coverage, pixel_anchors, pixel_weights,
                                    device=None):
    """NeuralNRT._C.compute_pixel_anchors_euclidean(graph_nodes, point_image, node_coverage, anchors, weights)."""
    d = _dev(device)
    a, w = pixel_anchors_euclidean_device(_t(graph_nodes, d, torch.float32), _t(point_image, d, torch.float32),
                                          node_coverage)
    _fill_inplace(pixel_anchors, a)
    _fill_inplace(pixel_weights, w)


def pixel_anchors_geodesic_device(node_to_vertex_distance, valid_nodes_mask, vertex_pixels, width, height,
                                  node_coverage):
    D = node_to_vertex_distance.contiguous().float()
    N, V = D.shape
    valid = valid_nodes_mask.reshape(-1).to(torch.int32).contiguous()
    vp = vertex_pixels.to(torch.int32).contiguous()
    assert vp.shape == (V, 2) and valid.shape[0] == N
    a = torch.empty((height, width, GRAPH_K), dtype=torch.int32, device=D.device)
    w = torch.empty((height, width, GRAPH_K), dtype=torch.float32, device=D.device)
    call("ofx_pixel_anchors_geodesic", ptr(D), ptr(valid), N, V, ptr(vp), int(width), int(height), float(node_coverage),
         ptr(a), ptr(w), stream_ptr())
    return a, w


def compute_pixel_anchors_geodesic(node_to_vertex_distance, valid_nodes_mask, vertices, vertex_pixels, pixel_anchors,
                                   pixel_weights, width, height, node_coverage, device=None):
    """NeuralNRT._C.compute_pixel_anchors_geodesic (argument order of the pybind binding, main.cpp)."""
    d = _dev(device)
    a, w = pixel_anchors_geodesic_device(_t(node_to_vertex_distance, d, torch.float32),
                                         _t(valid_nodes_mask, d, torch.int32), _t(vertex_pixels, d, torch.int32),
                                         width, height, node_coverage)
    _fill_inplace(pixel_anchors, a)
    _fill_inplace(pixel_weights, w)


def remap_anchors_device(anchors, id_map):
    """In place on a device int32 tensor; id_map: dense int32 (old id -> new id, -1 = no mapping).
    Raises IndexError (as std::map::at under pybind) if an anchor has no mapping."""
    assert anchors.dtype == torch.int32 and anchors.is_contiguous()
    m = id_map.to(device=anchors.device, dtype=torch.int32).contiguous()
    miss = torch.zeros(1, dtype=torch.int32, device=anchors.device)
    call("ofx_remap_anchors", ptr(anchors), anchors.numel(), ptr(m), m.numel(), ptr(miss), stream_ptr())
    if int(miss.item()):
        raise IndexError(f"update_pixel_anchors: {int(miss.item())} anchors without a node id mapping (map::at)")
    return anchors


def update_pixel_anchors(node_id_mapping, pixel_anchors, device=None):
    """NeuralNRT._C.update_pixel_anchors(node_id_mapping: dict old->new, pixel_anchors (H,W,K) i32) in place."""
    n_map = max(node_id_mapping) + 1 if node_id_mapping else 0
    dense = np.full(max(n_map, 1), -1, np.int32)
    for k, v in node_id_mapping.items():
        dense[k] = v
    a = _t(pixel_anchors, _dev(device), torch.int32)
    remap_anchors_device(a, torch.from_numpy(dense))
    pixel_anchors[...] = a.cpu().numpy()


def knn_device(points, nodes, k):
    """k nearest nodes -> (idx (P,k) i32, squared distances (P,k) f32), ascending (distance, id)."""
    pts = points.contiguous().float().reshape(-1, 3)
    nd = nodes.contiguous().float().reshape(-1, 3)
    P = pts.shape[0]
    idx = torch.empty((P, k), dtype=torch.int32, device=pts.device)
    d2 = torch.empty((P, k), dtype=torch.float32, device=pts.device)
    call("ofx_knn_points", ptr(pts), P, ptr(nd), nd.shape[0], int(k), ptr(idx), ptr(d2), stream_ptr())
    return idx, d2


# ------------------------------------------------------------------ ED-graph construction (§8(f) row 4)
class MeshGraph:
    """Device handle over a mesh (ofx_graph_create): vertex adjacency + the construction entry points.
    vertices (V,3) f32 / faces (F,3) i32 device tensors stay referenced by the handle."""

    def __init__(self, vertices, faces, device=None):
        from . import _lib
        d = _dev(device) if not isinstance(vertices, torch.Tensor) else vertices.device
        self.vertices = _t(vertices, d, torch.float32).reshape(-1, 3)
        self.faces = _t(faces, d, torch.int32).reshape(-1, 3)
        self.device = d
        self.nv, self.nf = self.vertices.shape[0], self.faces.shape[0]
        self._h = _lib.c_void_p()
        call("ofx_graph_create", ptr(self.vertices), self.nv, ptr(self.faces), self.nf, _lib.byref(self._h),
             stream_ptr())

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                _lib.lib.ofx_graph_destroy(h)
            except Exception:
                pass
            self._h = None

    def adjacency(self):
        from . import _lib
        n = _lib.c_int64()
        call("ofx_graph_adjacency", self._h, None, None, _lib.byref(n), stream_ptr())
        rp = torch.empty(self.nv + 1, dtype=torch.int32, device=self.device)
        col = torch.empty(max(1, n.value), dtype=torch.int32, device=self.device)
        call("ofx_graph_adjacency", self._h, ptr(rp), ptr(col), _lib.byref(n), stream_ptr())
        return rp, col[: n.value]

    def erode(self, n_iterations, min_neighbors):
        m = torch.empty(self.nv, dtype=torch.uint8, device=self.device)
        call("ofx_erode_mesh", self._h, int(n_iterations), int(min_neighbors), ptr(m), stream_ptr())
        return m.bool()

    def sample_nodes(self, non_eroded, node_coverage, use_only_non_eroded=True):
        """-> (node positions (n,3) f32, node vertex indices (n,) i32), ascending vertex order."""
        from . import _lib
        ne = None if non_eroded is None else _t(non_eroded, self.device, torch.uint8).reshape(-1)
        pos = torch.empty((max(1, self.nv), 3), dtype=torch.float32, device=self.device)
        idx = torch.empty(max(1, self.nv), dtype=torch.int32, device=self.device)
        n, rounds = _lib.c_int64(), _lib.c_int64()
        call("ofx_sample_nodes", self._h, ptr(ne), float(node_coverage), 1 if use_only_non_eroded else 0, ptr(pos),
             ptr(idx), _lib.byref(n), _lib.byref(rounds), stream_ptr())
        self.sample_rounds = int(rounds.value)
        return pos[: n.value], idx[: n.value]

    def edges_geodesic(self, node_indices, n_max_neighbors, node_coverage, allow_only_valid_vertices=True,
                       enforce_total_num_neighbors=True, valid_vertices=None, with_node_to_vertex=False):
        """-> (edges (N,K) i32, weights (N,K) f32, distances (N,K) f32, node_to_vertex (N,V) f32 or None)."""
        ni = _t(node_indices, self.device, torch.int32).reshape(-1)
        N, K = ni.shape[0], int(n_max_neighbors)
        kw = dict(device=self.device)
        E = torch.empty((N, K), dtype=torch.int32, **kw)
        W = torch.empty((N, K), dtype=torch.float32, **kw)
        D = torch.empty((N, K), dtype=torch.float32, **kw)
        n2v = torch.empty((N, self.nv), dtype=torch.float32, **kw) if with_node_to_vertex else None
        vv = None if valid_vertices is None else _t(valid_vertices, self.device, torch.uint8).reshape(-1)
        call("ofx_edges_geodesic", self._h, ptr(vv), ptr(ni), N, K, float(node_coverage),
             1 if allow_only_valid_vertices else 0, 1 if enforce_total_num_neighbors else 0, ptr(E), ptr(W), ptr(D),
             ptr(n2v), stream_ptr())
        from . import _lib
        nseq = _lib.c_int64()
        call("ofx_graph_geodesic_sequential", self._h, _lib.byref(nseq))
        self.geodesic_sequential = int(nseq.value)   # nodes settled by the sequential heap kernel
        return E, W, D, n2v


def downsample_device(nodes, node_coverage, device=None):
    """One level of EDGraph.create_graph_pyramid's down-sampling (embedded_deformation_graph.py:278-299) on the
    device -> (down_sample_idx, up_sample_idx) int lists, as the reference builds them."""
    from . import _lib
    dev = nodes.device if device is None and isinstance(nodes, torch.Tensor) else _dev(device)
    P = _t(nodes, dev, torch.float32).reshape(-1, 3).contiguous()
    n = P.shape[0]
    down = torch.empty(max(1, n), dtype=torch.int32, device=dev)
    up = torch.empty(max(1, n), dtype=torch.int32, device=dev)
    nd = _lib.c_int32()
    call("ofx_graph_downsample", ptr(P), n, float(node_coverage), ptr(down), ptr(up), _lib.byref(nd), stream_ptr())
    return down[: nd.value].cpu().tolist(), up[:n].cpu().tolist()


def edges_euclidean_device(nodes, n_max_neighbors):
    X = nodes.contiguous().float().reshape(-1, 3)
    E = torch.empty((X.shape[0], int(n_max_neighbors)), dtype=torch.int32, device=X.device)
    call("ofx_edges_euclidean", ptr(X), X.shape[0], int(n_max_neighbors), ptr(E), stream_ptr())
    return E


def node_edge_cleanup_device(edges, valid):
    E = edges.to(torch.int32).contiguous()
    vin = valid.reshape(-1).to(torch.uint8).contiguous()
    out = torch.empty_like(vin)
    call("ofx_node_edge_cleanup", ptr(E), E.shape[0], E.shape[1], ptr(vin), ptr(out), stream_ptr())
    return out.bool()


def clusters_device(edges):
    """-> (clusters (N,) i32, sizes list)."""
    from . import _lib
    E = edges.to(torch.int32).contiguous()
    N = E.shape[0]
    cl = torch.empty(max(1, N), dtype=torch.int32, device=E.device)
    sz = torch.empty(max(1, N), dtype=torch.int32, device=E.device)
    nc = _lib.c_int32()
    call("ofx_compute_clusters", ptr(E), N, E.shape[1], ptr(cl), ptr(sz), _lib.byref(nc), stream_ptr())
    return cl[:N], sz[: nc.value].cpu().tolist()


# ---- csrc call shapes (numpy in / numpy out, outputs resized or written in place) ----
def erode_mesh(vertexPositions, faceIndices, nIterations, minNeighbors, device=None):
    """NeuralNRT._C.erode_mesh -> non-eroded mask (V,1) bool."""
    g = MeshGraph(vertexPositions, faceIndices, device)
    return g.erode(nIterations, minNeighbors).cpu().numpy().reshape(-1, 1)


def sample_nodes(vertexPositions, nonErodedVertices, nodePositions, nodeIndices, nodeCoverage,
                 useOnlyNonErodedIndices=True, randomShuffle=True, device=None):
    """NeuralNRT._C.sample_nodes: outputs resized to (V,3) / (V,1) with the first n rows filled; returns n.
    randomShuffle visits the vertices in a random permutation (numpy generator; the reference seeds
    std::random_device, i.e. it is not reproducible either); EDGraph passes False."""
    P = np.ascontiguousarray(vertexPositions, np.float32).reshape(-1, 3)
    ne = np.asarray(nonErodedVertices).reshape(-1).astype(bool)
    V = P.shape[0]
    perm = np.random.default_rng().permutation(V) if randomShuffle else None
    if perm is not None:
        P, ne = P[perm], ne[perm]
    g = MeshGraph(P, np.zeros((0, 3), np.int32), device)
    pos, idx = g.sample_nodes(torch.from_numpy(ne.astype(np.uint8)), nodeCoverage, useOnlyNonErodedIndices)
    n = pos.shape[0]
    idx = idx.cpu().numpy()
    if perm is not None:
        idx = perm[idx].astype(np.int32)
    nodePositions.resize((V, 3), refcheck=False)
    nodeIndices.resize((V, 1), refcheck=False)
    nodePositions[:n] = pos.cpu().numpy()
    nodeIndices[:n, 0] = idx
    return n


def compute_edges_geodesic(vertexPositions, validVertices, faceIndices, nodeIndices, nMaxNeighbors, nodeCoverage,
                           graphEdges, graphEdgesWeights, graphEdgesDistances, nodeToVertexDistances,
                           allow_only_valid_vertices, enforce_total_num_neighbors, device=None):
    """NeuralNRT._C.compute_edges_geodesic: writes the four output arrays in place. Rows are fully written
    (-1 / 0 / 0 past the found neighbours, -1 for unvisited vertices): the values every reference call site
    pre-fills. Reaching an invalid vertex raises (the C++ calls exit(0))."""
    g = MeshGraph(vertexPositions, faceIndices, device)
    vv = np.asarray(validVertices).reshape(g.nv, -1)[:, 0].astype(np.uint8)
    E, W, D, n2v = g.edges_geodesic(np.asarray(nodeIndices).reshape(-1), nMaxNeighbors, nodeCoverage,
                                    allow_only_valid_vertices, enforce_total_num_neighbors,
                                    valid_vertices=torch.from_numpy(vv), with_node_to_vertex=True)
    graphEdges[...] = E.cpu().numpy()
    graphEdgesWeights[...] = W.cpu().numpy()
    graphEdgesDistances[...] = D.cpu().numpy()
    nodeToVertexDistances[...] = n2v.cpu().numpy()


def compute_edges_euclidean(nodePositions, nMaxNeighbors, device=None):
    """NeuralNRT._C.compute_edges_euclidean -> (N, K) int32."""
    return edges_euclidean_device(_t(nodePositions, _dev(device), torch.float32), nMaxNeighbors).cpu().numpy()


def node_and_edge_clean_up(graph_edges, valid_nodes_mask, device=None):
    """NeuralNRT._C.node_and_edge_clean_up: valid_nodes_mask (N,1) bool updated in place."""
    d = _dev(device)
    out = node_edge_cleanup_device(_t(graph_edges, d, torch.int32), _t(valid_nodes_mask, d, torch.uint8))
    valid_nodes_mask[...] = out.cpu().numpy().reshape(valid_nodes_mask.shape)


def compute_clusters(graph_edges, graph_clusters, device=None):
    """NeuralNRT._C.compute_clusters: graph_clusters (N,1) i32 written in place; returns the cluster sizes."""
    cl, sizes = clusters_device(_t(graph_edges, _dev(device), torch.int32))
    graph_clusters[...] = cl.cpu().numpy().reshape(graph_clusters.shape)
    return sizes
