"""ctypes binding of libofx.so (the C ABI declared in include/ofx.h).

torch is imported first so that libofx's NEEDED libamdhip64.so.7 resolves to the HIP runtime torch
already loaded (one runtime per process; device pointers from torch tensors are valid in libofx).
There is no fallback: if the library is missing or fails to load, importing this module raises.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede loading libofx)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("OFX_LIB") or os.path.join(_HERE, "libofx.so")   # OFX_LIB: tuning builds (tools/)

c_int32, c_int64, c_double, c_float, c_void_p = ctypes.c_int32, ctypes.c_int64, ctypes.c_double, ctypes.c_float, ctypes.c_void_p
P = ctypes.c_void_p  # device pointer


class VolumeDesc(ctypes.Structure):
    _fields_ = [("dim", c_int32 * 3), ("brick_x0", c_int32), ("brick_x1", c_int32), ("semantics", c_int32),
                ("origin", c_float * 3), ("_pad1", c_float), ("voxel_size", c_double), ("trunc_margin", c_double)]


class Camera(ctypes.Structure):
    _fields_ = [("fx", c_float), ("fy", c_float), ("cx", c_float), ("cy", c_float), ("width", c_int32),
                ("height", c_int32)]


class GnParams(ctypes.Structure):
    _fields_ = [("num_iter", c_int32), ("use_edge_weighting", c_int32), ("pcg_max_iter", c_int32), ("pcg_warm", c_int32),
                ("lambda_flow", c_double), ("lambda_depth", c_double), ("lambda_arap", c_double),
                ("lambda_motion", c_double), ("lm_factor", c_double), ("stop_loss_diff", c_double),
                ("pcg_tol", c_double), ("mode", c_int32), ("precond_every", c_int32),
                ("pcg_err_tol", c_double), ("precond_rot_tol", c_double), ("precond", c_int32), ("_pad1", c_int32)]


class GnProblem(ctypes.Structure):
    _fields_ = [("n_nodes", c_int32), ("n_matches", c_int32), ("n_neighbors", c_int32), ("_pad", c_int32),
                ("nodes", P), ("edges", P), ("edge_weights", P), ("target_node_pos", P), ("node_conf", P),
                ("src", P), ("anchors", P), ("weights", P), ("tgt", P), ("target_px", P), ("target_py", P),
                ("prev_rot", P), ("prev_trans", P), ("fx", c_float), ("fy", c_float), ("cx", c_float),
                ("cy", c_float)]


class GnResult(ctypes.Structure):
    _fields_ = [("rot", P), ("trans", P), ("status", P), ("loss_log", P)]


_SIGS = {
    "ofx_abi_version": [],
    "ofx_volume_num_slots": [P, P],
    "ofx_volume_reset": [P, P, P, P, P],
    "ofx_volume_to_dense": [P, P, P, P],
    "ofx_volume_from_dense": [P, P, P, P],
    "ofx_pack_color": [P, c_int32, c_int32, P, P],
    "ofx_skin_volume_bricks": [P, P, c_int32, c_double, c_int32, P, P, P],
    "ofx_skin_volume": [P, P, c_int32, c_double, c_int32, P, c_int32, P, P, P],
    "ofx_skin_palette": [P, c_int32, c_int32, c_int32, P, P, P, P],
    "ofx_skin_points": [P, c_int64, P, c_int32, c_double, c_int32, P, P, P, P],
    "ofx_skin_volume_to_dense": [P, P, c_int32, P, P, c_int32, P, P, P, P],
    "ofx_pack_nodes": [P, P, P, c_int32, P, P],
    "ofx_integrate": [P, P, P, P, c_int32, P, c_int32, c_int32, P, c_int32, P, P, c_double, P, P, P, P, P],
    "ofx_integrate_timing": [c_int32, P, P],
    "ofx_raycast": [P, P, P, P, P, c_float, c_float, P, P, P, P],
    "ofx_integrate_points": [P, P, P, P, P, P, P, c_int64, c_double, P, P, P, P, P],
    "ofx_integrate_palette": [P, P, P, P, P, c_int32, c_int32, P, c_int32, P, P, P, P, P, c_double, P, P, P, P, P],
    "ofx_integrate_palette_cull": [P, P, P, P, P, c_int32, c_int32, P, c_int32, P, P, P, P, P, c_double, P, P, P, P, P,
                                   P, P],
    "ofx_deform_points": [P, c_int64, P, P, P, c_int32, P, c_int32, c_int32, P, P],
    "ofx_deform_points_lbs": [P, c_int64, P, P, P, c_int32, P, P, c_int32, P, P],
    "ofx_visibility": [P, c_int64, P, P, c_double, P, P, P],
    "ofx_visibility_f32": [P, c_int64, P, P, c_double, P, P, P],
    "ofx_truncated_region": [P, P, c_double, P, P],
    "ofx_mesh_create": [P],
    "ofx_mesh_destroy": [P],
    "ofx_mesh_count": [P, P, P, P, c_double, c_int32, c_float, P, P, P],
    "ofx_mesh_count_range": [P, P, P, P, c_double, c_int32, c_float, c_int32, c_int32, P, P, P],
    "ofx_mesh_emit": [P, P, P, P, P, P, P],
    "ofx_mesh_finish": [P, P, P, c_int64, P, P, P],
    "ofx_backproject_depth": [P, c_int32, c_int32, c_int32, c_float, c_float, c_float, c_float, c_float, P, P],
    "ofx_depth_mesh_create": [P],
    "ofx_depth_mesh_destroy": [P],
    "ofx_depth_mesh_count": [P, P, c_int32, c_int32, c_float, P, P, P],
    "ofx_depth_mesh_emit": [P, P, P, P, P],
    "ofx_depth_to_pc": [P, P, c_int32, c_int32, c_double, c_double, c_double, c_double, P, P, P, P],
    "ofx_pixel_anchors_euclidean": [P, c_int32, P, c_int32, c_int32, c_float, P, P, P],
    "ofx_pixel_anchors_geodesic": [P, P, c_int32, c_int64, P, c_int32, c_int32, c_float, P, P, P],
    "ofx_remap_anchors": [P, c_int64, P, c_int32, P, P],
    "ofx_knn_points": [P, c_int64, P, c_int32, c_int32, P, P, P],
    "ofx_graph_create": [P, c_int64, P, c_int64, P, P],
    "ofx_graph_destroy": [P],
    "ofx_graph_adjacency": [P, P, P, P, P],
    "ofx_graph_geodesic_sequential": [P, P],
    "ofx_graph_downsample": [P, c_int32, c_double, P, P, P, P],
    "ofx_erode_mesh": [P, c_int32, c_int32, P, P],
    "ofx_sample_nodes": [P, P, c_float, c_int32, P, P, P, P, P],
    "ofx_edges_geodesic": [P, P, P, c_int32, c_int32, c_float, c_int32, c_int32, P, P, P, P, P],
    "ofx_edges_euclidean": [P, c_int32, c_int32, P, P],
    "ofx_node_edge_cleanup": [P, c_int32, c_int32, P, P, P],
    "ofx_compute_clusters": [P, c_int32, c_int32, P, P, P, P],
    "ofx_reduce_graph": [P, c_int32, c_int32, P, P, P, P, P, P, P, P, P, P, P, P],
    "ofx_gn_create": [c_int32, c_int32, P],
    "ofx_gn_destroy": [P],
    "ofx_gn_timing": [P, c_int32, P, P, P],
    "ofx_gn_info": [P, P],
    "ofx_gn_precond_info": [P, P],
    "ofx_gn_pcg_waves": [P, P],
    "ofx_gn_step_fused": [P, P],
    "ofx_gn_stopped": [P, P],
    "ofx_gn_stats": [P, P, c_int32],
    "ofx_gn_row_order": [P, P, c_int32],
    "ofx_gn_setup": [P, P, P, P, P],
    "ofx_gn_linearize": [P, c_int32, c_int32, c_int32, c_int32, P, P, P],
    "ofx_gn_step": [P, c_int32, P, P, P],
    "ofx_gn_finish": [P, P, P],
    "ofx_gn_solve": [P, P, P, P, P],
    "ofx_gn_prepare": [P, P, P, P],
    "ofx_gn_prepare_after": [P, P, P, P, P, c_int32],
    "ofx_gn_prepare_wait": [P, P],
    "ofx_gn_prefetch_stats": [P, P, P],
    "ofx_gn_share_history": [P, P],
    "ofx_gn_set_idle_hook": [P, P, P],
}


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libofx.so not built at {LIB_PATH}: run `python -m occlusionfusion_amd.build` "
                          "(no CPU fallback exists for the fusion hot path)")
    lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    for name, argtypes in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = c_int32
    lib.ofx_last_error.argtypes = []
    lib.ofx_last_error.restype = ctypes.c_char_p
    return lib


lib = _load()
EXPORTED = tuple(_SIGS) + ("ofx_last_error",)


PALETTE = 64   # OFX_PALETTE (include/ofx.h)


class OfxError(RuntimeError):
    pass


def check(status, what=""):
    if status != 0:
        msg = lib.ofx_last_error().decode(errors="replace")
        raise OfxError(f"{what or 'libofx'} failed (status {status}): {msg}")


def call(name, *args):
    check(getattr(lib, name)(*args), name)


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream_ptr(stream=None):
    s = torch.cuda.current_stream() if stream is None else stream
    return ctypes.c_void_p(s.cuda_stream)


def byref(x):
    return ctypes.byref(x)
