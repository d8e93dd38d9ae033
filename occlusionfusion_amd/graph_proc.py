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
