"""The reference's on-disk formats for graphs and per-pixel images (utils/utils.py:205-383): a native-endian
uint32 header (counts / dims) followed by the row-major payload. numpy fromfile/tofile, no pickle.

  nodes / node deformations: [N] + f32[N*3]       edges: [N, K] + i32[N*K]     edge weights: [N, K] + f32
  clusters: [N, 1] + i32[N]                       float / int image (X,Y,Z): [Z, Y, X] + payload
The volume checkpoint (TSDFVolume.save_volume / load_volume) is the stacked (3,Dx,Dy,Dz) array of
tsdf.py:682-702 written with np.save (the reference pickles it; pickles are never loaded here).
"""
import numpy as np

_U32 = np.dtype("=u4")


def _write(filename, header, arr, dtype):
    with open(filename, "wb") as f:
        np.asarray(header, _U32).tofile(f)
        np.ascontiguousarray(arr, dtype).tofile(f)


def _read(filename, n_header, dtype, shape_of):
    with open(filename, "rb") as f:
        h = np.fromfile(f, _U32, n_header)
        if h.size != n_header:
            raise ValueError(f"{filename}: truncated header")
        shape = shape_of(h)
        data = np.fromfile(f, dtype, int(np.prod(shape)))
    if data.size != int(np.prod(shape)):
        raise ValueError(f"{filename}: truncated payload")
    return data.reshape(shape)


def save_graph_nodes(filename, nodes):
    assert nodes.ndim == 2 and nodes.shape[1] == 3
    _write(filename, [nodes.shape[0]], nodes, np.float32)


def load_graph_nodes(filename):
    return _read(filename, 1, np.dtype("=f4"), lambda h: (int(h[0]), 3))


save_graph_node_deformations = save_graph_nodes
load_graph_node_deformations = load_graph_nodes


def save_graph_edges(filename, edges):
    assert edges.ndim == 2
    _write(filename, edges.shape, edges, np.int32)


def load_graph_edges(filename):
    return _read(filename, 2, np.dtype("=i4"), lambda h: (int(h[0]), int(h[1])))


def save_graph_edges_weights(filename, w):
    assert w.ndim == 2
    _write(filename, w.shape, w, np.float32)


def load_graph_edges_weights(filename):
    return _read(filename, 2, np.dtype("=f4"), lambda h: (int(h[0]), int(h[1])))


def save_graph_clusters(filename, clusters):
    assert clusters.ndim == 2
    _write(filename, clusters.shape, clusters, np.int32)


def load_graph_clusters(filename):
    return _read(filename, 2, np.dtype("=i4"), lambda h: (int(h[0]), 1))


def save_float_image(filename, image):
    assert image.ndim == 3
    _write(filename, image.shape[::-1], image, np.float32)


def load_float_image(filename):
    return _read(filename, 3, np.dtype("=f4"), lambda h: (int(h[2]), int(h[1]), int(h[0])))


def save_int_image(filename, image):
    assert image.ndim == 3
    _write(filename, image.shape[::-1], image, np.int32)


def load_int_image(filename):
    return _read(filename, 3, np.dtype("=i4"), lambda h: (int(h[2]), int(h[1]), int(h[0])))
