"""Correspondence front-end plumbing on the device, behind the reference's own names.

  backproject_depth          utils/image_proc.py:335-349 -> csrc backproject_depth_float / _ushort
                             (csrc/cpu/image_proc.cpp:351-401)                       -> ofx_backproject_depth
  compute_mesh_from_depth    NeuralNRT._C.compute_mesh_from_depth (csrc/cpu/image_proc.cpp:405-545), same
                             call shape as its callers use it (embedded_deformation_graph.py:136-145,
                             warpfield.py:160-170): outputs are zero-size arrays resized in place
                                                                                     -> ofx_depth_mesh_*
  depth_2_pc / target cloud  NonRigidICP/model/geometry.py:44-59 + Registration.optimize's masked cloud and
                             map_pixel_to_pcd (registration_fusion.py:104-109,388-395) -> ofx_depth_to_pc

Results are bit-identical to the reference C++ (backproject, mesh) and to the numpy float64 expression
rounded to f32 (depth_2_pc): tests/test_gpu_frontend.py. There is no CPU fallback.
"""
import numpy as np
import torch

from . import _lib
from ._lib import byref, call, ptr, stream_ptr

_handles = {}


def _handle(device):
    """Per-device scratch handle (ofx_depth_mesh_create) shared by the mesh and point-cloud entry points."""
    idx = torch.device(device).index or 0
    h = _handles.get(idx)
    if h is None:
        h = _lib.c_void_p()
        with torch.cuda.device(idx):
            call("ofx_depth_mesh_create", byref(h))
        _handles[idx] = h
    return h


def _device(device):
    return torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())


def backproject_depth_device(depth, fx, fy, cx, cy, normalizer=1000.0, out=None):
    """depth: (H, W) float32 metres or uint16/int16 (scaled by 1/normalizer) device tensor -> (3, H, W) f32."""
    assert depth.dim() == 2, "depth image must be (H, W)"
    H, W = depth.shape
    is_u16 = depth.dtype != torch.float32
    if is_u16:
        assert depth.dtype in (torch.uint16, torch.int16), "integer depth must be 16-bit (uint16 mm)"
    d = depth.contiguous()
    if out is None:
        out = torch.zeros((3, H, W), dtype=torch.float32, device=d.device)
    call("ofx_backproject_depth", ptr(d), 1 if is_u16 else 0, H, W, float(fx), float(fy), float(cx), float(cy),
         float(normalizer), ptr(out), stream_ptr())
    return out


def backproject_depth(depth_image, fx, fy, cx, cy, normalizer=1000.0, device=None):
    """utils/image_proc.py:335-349: (H, W) numpy depth -> (3, H, W) float32 point image."""
    assert len(depth_image.shape) == 2
    dev = _device(device)
    if depth_image.dtype == np.float32:
        d = torch.from_numpy(np.ascontiguousarray(depth_image)).to(dev)
    else:   # the reference hands every non-f32 image to the ushort binding
        d = torch.from_numpy(np.ascontiguousarray(depth_image.astype(np.uint16)).view(np.int16)).to(dev)
    return backproject_depth_device(d, fx, fy, cx, cy, normalizer).cpu().numpy()


def compute_mesh_from_depth_device(point_image, max_triangle_distance, with_pixels=True):
    """point_image (3, H, W) f32 device tensor -> dict(vertices (V,3) f32, vertex_pixels (V,2) i32 [x, y],
    faces (F,3) i32), numbered as the sequential C++ does. One host sync (the output size)."""
    assert point_image.dim() == 3 and point_image.shape[0] == 3, "point image must be (3, H, W)"
    p = point_image.contiguous()
    if p.dtype != torch.float32:
        p = p.float()
    _, H, W = p.shape
    h = _handle(p.device)
    nv, nf = _lib.c_int64(), _lib.c_int64()
    call("ofx_depth_mesh_count", h, ptr(p), H, W, float(max_triangle_distance), byref(nv), byref(nf), stream_ptr())
    V, F = int(nv.value), int(nf.value)
    out = {"vertices": torch.empty((V, 3), dtype=torch.float32, device=p.device),
           "vertex_pixels": torch.empty((V, 2), dtype=torch.int32, device=p.device) if with_pixels else None,
           "faces": torch.empty((F, 3), dtype=torch.int32, device=p.device)}
    call("ofx_depth_mesh_emit", h, ptr(out["vertices"]), ptr(out["vertex_pixels"]), ptr(out["faces"]), stream_ptr())
    return out


def compute_mesh_from_depth(point_image, max_triangle_distance, vertex_positions, vertex_pixels, face_indices,
                            device=None):
    """NeuralNRT._C.compute_mesh_from_depth signature: numpy point image (3, H, W) and zero-size output arrays
    that are resized in place (like the pybind binding's `resize`, image_proc.cpp:523-526). As in the C++,
    the outputs stay untouched unless both vertex and face counts are positive."""
    p = torch.from_numpy(np.ascontiguousarray(point_image, np.float32)).to(_device(device))
    m = compute_mesh_from_depth_device(p, max_triangle_distance)
    V, F = m["vertices"].shape[0], m["faces"].shape[0]
    if V > 0 and F > 0:
        for arr, t, shape in ((vertex_positions, m["vertices"], (V, 3)), (vertex_pixels, m["vertex_pixels"], (V, 2)),
                              (face_indices, m["faces"], (F, 3))):
            arr.resize(shape, refcheck=False)
            arr[...] = t.cpu().numpy()
    return V, F


def depth_2_pc_device(depth, intrin, with_map=True):
    """Registration.optimize target cloud (registration_fusion.py:104-109): depth (H, W) f32 device tensor,
    intrin 3x3 (fx = K[0,0], fy = K[1,1], cx = K[0,2], cy = K[1,2]) or (fx, fy, cx, cy) ->
    (points (P,3) f32 of the pixels with depth > 0 in row-major order, pix_2_pcd (H,W) int64 or None)."""
    K = np.asarray(intrin, np.float64)
    fx, fy, cx, cy = (K[0, 0], K[1, 1], K[0, 2], K[1, 2]) if K.shape == (3, 3) else tuple(K.reshape(-1)[:4])
    d = depth.contiguous()
    assert d.dtype == torch.float32 and d.dim() == 2
    H, W = d.shape
    pts = torch.empty((H * W, 3), dtype=torch.float32, device=d.device)
    pmap = torch.empty((H, W), dtype=torch.int64, device=d.device) if with_map else None
    n = torch.empty(1, dtype=torch.int32, device=d.device)
    call("ofx_depth_to_pc", _handle(d.device), ptr(d), H, W, float(fx), float(fy), float(cx), float(cy), ptr(pts),
         ptr(pmap), ptr(n), stream_ptr())
    return pts[: int(n.item())], pmap


def depth_2_pc(depth, intrin, device=None):
    """numpy convenience: -> (points (P,3) f32, pix_2_pcd (H,W) int64)."""
    d = torch.from_numpy(np.ascontiguousarray(depth, np.float32)).to(_device(device))
    pts, pmap = depth_2_pc_device(d, intrin)
    return pts.cpu().numpy(), pmap.cpu().numpy()
