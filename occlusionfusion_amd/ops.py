"""PyTorch-ROCm custom operators over the libofx C ABI: `torch.ops.ofx.*` (torch.library).

The shims (TSDFVolume, WarpField, GaussNewtonSolver) call these operators, so the fusion hot path is
visible to the dispatcher, to FakeTensor / meta tracing and to graph capture with the kernels still the
hand-written HIP ones in libofx.so. Conventions:

* every operator is registered for the CUDA (= HIP) dispatch key only: CPU tensors raise
  NotImplementedError ("no kernel for CPU") — there is no CPU fallback;
* work is enqueued on torch's current stream of the tensors' device, asynchronously (no host sync);
* in-place outputs are declared in the schema (`Tensor(a!)`), so functionalisation sees the mutation;
* the GN operators take the solver handle (an `int`, the C pointer) and a one-element `state` tensor that
  they declare mutated: the handle's scratch (warm-start ring, preconditioner, row order) is hidden state,
  and the declared mutation keeps two solves on one handle ordered under any graph transformation;
* every operator has a fake (meta) kernel giving output shapes and dtypes without a device.

Registration is the low-level `torch.library.Library` form (schema inferred from the Python signature exactly
as `torch.library.custom_op` would, CUDA kernel + fake kernel) rather than the `custom_op` decorator: the
decorator's Python-side autograd / mutation wrapping costs ≈ 50 µs per call on the host, and the fusion loop
issues two of these calls per frame on its critical path (measured: 69 vs 19 µs per 18-argument call).

Reference call sites these operators replace: TSDFVolume.integrate (fusion_with_occlusion/tsdf.py:378-494),
WarpField.skin / deform (warpfield.py:83-129, 270-305, 369-380), DeformNet.optimize (model/model.py:222-859).
"""
from typing import List, Optional, Tuple

import torch
from torch import Tensor

from . import _lib
from ._lib import byref, call, ptr, stream_ptr

_NS = "ofx"
_LIB = torch.library.Library(_NS, "FRAGMENT")


class _Op:
    """One registered operator: `fn` is its CUDA kernel; `register_fake` attaches the meta kernel."""

    def __init__(self, name, fn):
        self.name, self.fn = name, fn

    def __call__(self, *args):
        return getattr(torch.ops.ofx, self.name)(*args)

    def register_fake(self, fake):
        torch.library.register_fake(f"{_NS}::{self.name}", fake, lib=_LIB)
        return fake


def _op(name, mutates_args):
    def deco(fn):
        _LIB.define(name + torch.library.infer_schema(fn, mutates_args=mutates_args))
        _LIB.impl(name, fn, "CUDA")
        return _Op(name, fn)
    return deco


def _volume_desc(dims, brick_range, origin, voxel_size, trunc_margin, semantics):
    d = _lib.VolumeDesc()
    d.dim[:] = [int(x) for x in dims]
    d.brick_x0, d.brick_x1 = int(brick_range[0]), int(brick_range[1])
    d.origin[:] = [float(x) for x in origin]
    d.voxel_size, d.trunc_margin, d.semantics = float(voxel_size), float(trunc_margin), int(semantics)
    return d


def _camera(intr, height, width):
    c = _lib.Camera()
    c.fx, c.fy, c.cx, c.cy = (float(v) for v in intr[:4])
    c.height, c.width = int(height), int(width)
    return c


def _stream(t):
    return stream_ptr(torch.cuda.current_stream(t.device))


# --------------------------------------------------------------------------------------------- integrate
@_op("integrate", mutates_args=("tsdf", "weight", "color", "n_updated"))
def integrate(tsdf: Tensor, weight: Tensor, color: Optional[Tensor], n_updated: Optional[Tensor], depth: Tensor,
              color_im: Optional[Tensor], dims: List[int], brick_range: List[int], origin: List[float],
              voxel_size: float, trunc_margin: float, semantics: int, intr: List[float], obs_weight: float,
              packed_nodes: Optional[Tensor], n_nodes: int, k: int, brick_list: Optional[Tensor], n_list: int,
              anchors: Optional[Tensor], weights: Optional[Tensor], pal_ids: Optional[Tensor],
              pal_n: Optional[Tensor], local: Optional[Tensor]) -> None:
    """TSDFVolume.integrate's device work (tsdf.py:378-494): source frame when packed_nodes is None
    (ofx_integrate warp=0), else the fused skin-cache ED warp + integrate of the listed bricks — through the
    LDS node palette when pal_ids is given (ofx_integrate_palette), with global node gathers otherwise."""
    desc = _volume_desc(dims, brick_range, origin, voxel_size, trunc_margin, semantics)
    cam = _camera(intr, depth.shape[0], depth.shape[1])
    s = _stream(tsdf)
    if packed_nodes is None:   # source frame; brick_list: a hash shard's own bricks (None: all of the shard)
        call("ofx_integrate", byref(desc), byref(cam), ptr(depth), ptr(color_im), 0, None, 0, 1, ptr(brick_list),
             n_list, None, None, float(obs_weight), ptr(tsdf), ptr(weight), ptr(color), ptr(n_updated), s)
    elif pal_ids is not None:
        call("ofx_integrate_palette", byref(desc), byref(cam), ptr(depth), ptr(color_im), ptr(packed_nodes), n_nodes, k,
             ptr(brick_list), n_list, ptr(anchors), ptr(weights), ptr(pal_ids), ptr(pal_n), ptr(local),
             float(obs_weight), ptr(tsdf), ptr(weight), ptr(color), ptr(n_updated), s)
    else:
        call("ofx_integrate", byref(desc), byref(cam), ptr(depth), ptr(color_im), 1, ptr(packed_nodes), n_nodes, k,
             ptr(brick_list), n_list, ptr(anchors), ptr(weights), float(obs_weight), ptr(tsdf), ptr(weight),
             ptr(color), ptr(n_updated), s)


@integrate.register_fake
def _(tsdf, weight, color, n_updated, depth, color_im, dims, brick_range, origin, voxel_size, trunc_margin, semantics,
      intr, obs_weight, packed_nodes, n_nodes, k, brick_list, n_list, anchors, weights, pal_ids, pal_n, local):
    return None


@_op("integrate_points", mutates_args=("tsdf", "weight", "color", "n_updated"))
def integrate_points(tsdf: Tensor, weight: Tensor, color: Optional[Tensor], n_updated: Optional[Tensor],
                     depth: Tensor, color_im: Optional[Tensor], dims: List[int], brick_range: List[int],
                     origin: List[float], voxel_size: float, trunc_margin: float, semantics: int, intr: List[float],
                     obs_weight: float, points: Tensor, voxel_ids: Tensor, valid: Optional[Tensor]) -> None:
    """TSDFVolume.integrate of given (already deformed) points into the voxels `voxel_ids` (C-order ids,
    distinct): tsdf.py:442-494 with pts from WarpField.deform_tsdf (warpfield.py:369-380)."""
    desc = _volume_desc(dims, brick_range, origin, voxel_size, trunc_margin, semantics)
    cam = _camera(intr, depth.shape[0], depth.shape[1])
    call("ofx_integrate_points", byref(desc), byref(cam), ptr(depth), ptr(color_im), ptr(points), ptr(voxel_ids),
         ptr(valid), points.shape[0], float(obs_weight), ptr(tsdf), ptr(weight), ptr(color), ptr(n_updated),
         _stream(tsdf))


@integrate_points.register_fake
def _(tsdf, weight, color, n_updated, depth, color_im, dims, brick_range, origin, voxel_size, trunc_margin, semantics,
      intr, obs_weight, points, voxel_ids, valid):
    return None


@_op("raycast", mutates_args=())
def raycast(tsdf: Tensor, weight: Tensor, color: Optional[Tensor], dims: List[int], origin: List[float],
            voxel_size: float, trunc_margin: float, intr: List[float], height: int, width: int, z_near: float,
            z_far: float) -> Tuple[Tensor, Tensor, Tensor]:
    """Depth (H,W), normals (H,W,3) and packed colours (H,W) of the fused surface seen from the camera
    (ofx_raycast; new capability, no reference twin)."""
    nbx = (int(dims[0]) + 7) // 8
    desc = _volume_desc(dims, [0, nbx], origin, voxel_size, trunc_margin, 0)
    cam = _camera(intr, height, width)
    depth = torch.empty((height, width), dtype=torch.float32, device=tsdf.device)
    normals = torch.empty((height, width, 3), dtype=torch.float32, device=tsdf.device)
    colors = torch.empty((height, width), dtype=torch.float32, device=tsdf.device)
    call("ofx_raycast", byref(desc), byref(cam), ptr(tsdf), ptr(weight), ptr(color), float(z_near), float(z_far),
         ptr(depth), ptr(normals), ptr(colors), _stream(tsdf))
    return depth, normals, colors


@raycast.register_fake
def _(tsdf, weight, color, dims, origin, voxel_size, trunc_margin, intr, height, width, z_near, z_far):
    return (tsdf.new_empty((height, width)), tsdf.new_empty((height, width, 3)), tsdf.new_empty((height, width)))


# --------------------------------------------------------------------------------------------- skinning
@_op("skin_points", mutates_args=())
def skin_points(points: Tensor, nodes: Tensor, node_coverage: float, k: int) -> Tuple[Tensor, Tensor, Tensor]:
    """WarpField.skin (warpfield.py:83-129): k nearest nodes, exp(-d²/2σ²) weights normalised by Σ + 1e-6,
    4σ cut-off -> (anchors int32 (P,k), weights f32 (P,k), valid bool (P,))."""
    P = points.shape[0]
    anchors = torch.empty((P, k), dtype=torch.int32, device=points.device)
    weights = torch.empty((P, k), dtype=torch.float32, device=points.device)
    valid = torch.empty(P, dtype=torch.uint8, device=points.device)
    call("ofx_skin_points", ptr(points), P, ptr(nodes), nodes.shape[0], float(node_coverage), int(k), ptr(anchors),
         ptr(weights), ptr(valid), _stream(points))
    return anchors, weights, valid.bool()


@skin_points.register_fake
def _(points, nodes, node_coverage, k):
    P = points.shape[0]
    return (points.new_empty((P, k), dtype=torch.int32), points.new_empty((P, k), dtype=torch.float32),
            points.new_empty((P,), dtype=torch.bool))


# --------------------------------------------------------------------------------------------- warp
@_op("deform_points", mutates_args=())
def deform_points(points: Tensor, anchors: Tensor, weights: Tensor, valid: Optional[Tensor], packed_nodes: Tensor,
                  normals: bool) -> Tensor:
    """ED_warp (NonRigidICP/model/geometry.py:9-25) of points with their skin; normals=True: the rotation-only
    blend of WarpField.deform_normals (warpfield.py:312-345). Points with valid == 0 keep their position."""
    out = torch.empty_like(points)
    v = None if valid is None else valid.to(torch.uint8)
    call("ofx_deform_points", ptr(points), points.shape[0], ptr(anchors), ptr(weights), ptr(v), anchors.shape[1],
         ptr(packed_nodes), packed_nodes.shape[0], 1 if normals else 0, ptr(out), _stream(points))
    return out


@deform_points.register_fake
def _(points, anchors, weights, valid, packed_nodes, normals):
    return torch.empty_like(points)


# --------------------------------------------------------------------------------------------- Gauss-Newton
def _gn_problem(nodes, edges, edge_weights, tpos, conf, src, anchors, weights, tgt, target_px, target_py, prev_rot,
                prev_trans, intr):
    pb = _lib.GnProblem()
    pb.n_nodes, pb.n_matches, pb.n_neighbors = nodes.shape[0], src.shape[0], edges.shape[1]
    pb.nodes, pb.edges, pb.edge_weights = ptr(nodes), ptr(edges), ptr(edge_weights)
    pb.target_node_pos, pb.node_conf = ptr(tpos), ptr(conf)
    pb.src, pb.anchors, pb.weights, pb.tgt = ptr(src), ptr(anchors), ptr(weights), ptr(tgt)
    pb.target_px, pb.target_py = ptr(target_px), ptr(target_py)
    pb.prev_rot, pb.prev_trans = ptr(prev_rot), ptr(prev_trans)
    pb.fx, pb.fy, pb.cx, pb.cy = (float(v) for v in intr[:4])
    return pb


def _gn_params(fparams, iparams):
    """fparams = [lambda_flow, lambda_depth, lambda_arap, lambda_motion, lm_factor, stop_loss_diff, pcg_tol,
    pcg_err_tol, precond_rot_tol]; iparams = [num_iter, use_edge_weighting, pcg_max_iter, pcg_warm, mode,
    precond_every(, precond: OFX_PRECOND_CLUSTER 0 / OFX_PRECOND_SCHWARZ 1, default 0)]."""
    p = _lib.GnParams()
    (p.lambda_flow, p.lambda_depth, p.lambda_arap, p.lambda_motion, p.lm_factor, p.stop_loss_diff,
     p.pcg_tol, p.pcg_err_tol, p.precond_rot_tol) = (float(v) for v in fparams)
    p.num_iter, p.use_edge_weighting, p.pcg_max_iter, p.pcg_warm, p.mode, p.precond_every = (int(v) for v in iparams[:6])
    p.precond = int(iparams[6]) if len(iparams) > 6 else 0
    return p


def _gn_outputs(N, num_iter, device):
    # k_finish writes every element (status and all num_iter loss rows): no fill kernels
    return (torch.empty((N, 3, 3), device=device), torch.empty((N, 3), device=device),
            torch.empty(5, dtype=torch.int32, device=device),
            torch.empty((num_iter, 4), dtype=torch.float64, device=device))


def _gn_result(out):
    r = _lib.GnResult()
    r.rot, r.trans, r.status, r.loss_log = (ptr(t) for t in out)
    return r


@_op("gn_solve", mutates_args=("state",))
def gn_solve(state: Tensor, handle: int, nodes: Tensor, edges: Tensor, edge_weights: Tensor, tpos: Tensor,
             conf: Tensor, src: Tensor, anchors: Tensor, weights: Tensor, tgt: Tensor, target_px: Optional[Tensor],
             target_py: Optional[Tensor], prev_rot: Optional[Tensor], prev_trans: Optional[Tensor],
             intr: List[float], fparams: List[float], iparams: List[int]) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """DeformNet.optimize (model/model.py:222-859) for one batch item on the device: -> (node_rotations (N,3,3),
    node_translations (N,3), status int32[5] = [valid, GN steps, PCG iterations, ill-posed, GN steps whose PCG hit
    pcg_max_iter], loss f64[num_iter,4])."""
    pb = _gn_problem(nodes, edges, edge_weights, tpos, conf, src, anchors, weights, tgt, target_px, target_py,
                     prev_rot, prev_trans, intr)
    prm = _gn_params(fparams, iparams)
    out = _gn_outputs(nodes.shape[0], int(iparams[0]), nodes.device)
    call("ofx_gn_solve", _lib.c_void_p(handle), byref(pb), byref(prm), byref(_gn_result(out)), _stream(nodes))
    return out


@gn_solve.register_fake
def _(state, handle, nodes, edges, edge_weights, tpos, conf, src, anchors, weights, tgt, target_px, target_py,
      prev_rot, prev_trans, intr, fparams, iparams):
    N = nodes.shape[0]
    return (nodes.new_empty((N, 3, 3)), nodes.new_empty((N, 3)), nodes.new_empty((5,), dtype=torch.int32),
            nodes.new_empty((int(iparams[0]), 4), dtype=torch.float64))


@_op("gn_prepare", mutates_args=("state",))
def gn_prepare(state: Tensor, handle: int, nodes: Tensor, edges: Tensor, edge_weights: Tensor, tpos: Tensor,
               conf: Tensor, src: Tensor, anchors: Tensor, weights: Tensor, tgt: Tensor, target_px: Optional[Tensor],
               target_py: Optional[Tensor], intr: List[float], fparams: List[float], iparams: List[int],
               trigger: int = 0, trigger_step: int = 0) -> None:
    """ofx_gn_prepare: prefetch the setup of the next gn_solve on this handle (host thread + the handle's own
    stream, ordered after the current stream's work); returns at once. The tensors must stay alive and
    unchanged until that solve. trigger != 0 (ofx_gn_prepare_after): the setup starts when the next gn_solve on
    handle `trigger` reaches GN step trigger_step (or returns)."""
    pb = _gn_problem(nodes, edges, edge_weights, tpos, conf, src, anchors, weights, tgt, target_px, target_py,
                     None, None, intr)
    prm = _gn_params(fparams, iparams)
    if trigger:
        call("ofx_gn_prepare_after", _lib.c_void_p(handle), byref(pb), byref(prm), _stream(nodes),
             _lib.c_void_p(trigger), int(trigger_step))
    else:
        call("ofx_gn_prepare", _lib.c_void_p(handle), byref(pb), byref(prm), _stream(nodes))


@gn_prepare.register_fake
def _(state, handle, nodes, *rest):
    return None


@_op("gn_setup", mutates_args=("state",))
def gn_setup(state: Tensor, handle: int, nodes: Tensor, edges: Tensor, edge_weights: Tensor, tpos: Tensor,
             conf: Tensor, src: Tensor, anchors: Tensor, weights: Tensor, tgt: Tensor, target_px: Optional[Tensor],
             target_py: Optional[Tensor], prev_rot: Optional[Tensor], prev_trans: Optional[Tensor],
             intr: List[float], fparams: List[float], iparams: List[int]) -> Tensor:
    """ofx_gn_setup: upload the problem and build the JᵀJ block pattern -> int64[2] (host) = [JᵀJ blocks, PCG
    rows] (one stream sync, as the C call)."""
    pb = _gn_problem(nodes, edges, edge_weights, tpos, conf, src, anchors, weights, tgt, target_px, target_py,
                     prev_rot, prev_trans, intr)
    prm = _gn_params(fparams, iparams)
    nnz = _lib.c_int64()
    h = _lib.c_void_p(handle)
    call("ofx_gn_setup", h, byref(pb), byref(prm), byref(nnz), _stream(nodes))
    info = (_lib.c_int64 * 5)()
    call("ofx_gn_info", h, info)
    return torch.tensor([nnz.value, info[4]], dtype=torch.int64)


@gn_setup.register_fake
def _(state, handle, nodes, *rest):
    return torch.empty(2, dtype=torch.int64, device="cpu")


@_op("gn_linearize", mutates_args=("state", "A", "rhs"))
def gn_linearize(state: Tensor, handle: int, it: int, m0: int, m1: int, regularizers: bool, A: Tensor,
                 rhs: Tensor) -> None:
    """One GN step's JᵀJ (BSR 6x6 f64 blocks, A) and -Jᵀr (rhs, + loss² tail) over matches [m0, m1), plus the
    ARAP / motion rows and the LM damping when `regularizers` (model.py:415-662)."""
    call("ofx_gn_linearize", _lib.c_void_p(handle), int(it), int(m0), int(m1), 1 if regularizers else 0, ptr(A),
         ptr(rhs), _stream(A))


@gn_linearize.register_fake
def _(state, handle, it, m0, m1, regularizers, A, rhs):
    return None


@_op("gn_step", mutates_args=("state",))
def gn_step(state: Tensor, handle: int, it: int, A: Tensor, rhs: Tensor) -> None:
    """Solve A x = rhs (PCG) and take the GN step (loss rule, kornia exp map, R ← exp(x)·R, t += x; model.py:
    694-748)."""
    call("ofx_gn_step", _lib.c_void_p(handle), int(it), ptr(A), ptr(rhs), _stream(A))


@gn_step.register_fake
def _(state, handle, it, A, rhs):
    return None


@_op("gn_finish", mutates_args=("state",))
def gn_finish(state: Tensor, handle: int, n_nodes: int, num_iter: int) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """Results of the stepped solve (ofx_gn_finish): as gn_solve's outputs."""
    out = _gn_outputs(n_nodes, num_iter, state.device)
    call("ofx_gn_finish", _lib.c_void_p(handle), byref(_gn_result(out)), _stream(state))
    return out


@gn_finish.register_fake
def _(state, handle, n_nodes, num_iter):
    return (state.new_empty((n_nodes, 3, 3), dtype=torch.float32), state.new_empty((n_nodes, 3), dtype=torch.float32),
            state.new_empty((5,), dtype=torch.int32), state.new_empty((num_iter, 4), dtype=torch.float64))


OPS = ("integrate", "integrate_points", "raycast", "skin_points", "deform_points", "gn_solve", "gn_prepare", "gn_setup",
       "gn_linearize", "gn_step", "gn_finish")
