"""GPU: the torch.ops.ofx.* operators (ops.py) give exactly what the direct C-ABI calls give on the same
inputs (bit for bit), pass torch.library.opcheck (schema, fake kernel and dispatch consistency), and run
on torch's current stream."""
import ctypes
import os

import numpy as np
import pytest
import torch

from occlusionfusion_amd import _lib
from occlusionfusion_amd._lib import byref, call, ptr, stream_ptr

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def small(golden_dir):
    return np.load(os.path.join(golden_dir, "integrate_small.npz"), allow_pickle=False)


def _skin_direct(pts, nodes, cov, K):
    P = pts.shape[0]
    a = torch.empty((P, K), dtype=torch.int32, device=pts.device)
    w = torch.empty((P, K), dtype=torch.float32, device=pts.device)
    v = torch.empty(P, dtype=torch.uint8, device=pts.device)
    call("ofx_skin_points", ptr(pts), P, ptr(nodes), nodes.shape[0], cov, K, ptr(a), ptr(w), ptr(v), stream_ptr())
    return a, w, v.bool()


def test_skin_and_deform_ops_equal_direct_calls(cuda, small):
    g = small
    rng = np.random.default_rng(0)
    pts = torch.from_numpy((rng.random((50000, 3)) * [0.8, 0.6, 0.8] + [-0.4, -0.33, 0.95]).astype(np.float32)).to(cuda)
    nodes = torch.from_numpy(g["nodes"]).to(cuda)
    cov = float(g["node_coverage"])
    a0, w0, v0 = _skin_direct(pts, nodes, cov, 4)
    a1, w1, v1 = torch.ops.ofx.skin_points(pts, nodes, cov, 4)
    assert torch.equal(a0, a1) and torch.equal(w0, w1) and torch.equal(v0, v1)
    from occlusionfusion_amd import EDGraph, WarpField, TSDFVolume
    from occlusionfusion_amd.synthetic import euclidean_edges
    vol = TSDFVolume.from_grid(g["origin"], float(g["voxel_size"]), g["dims"], tuple(g["intr"]), device=cuda)
    e, ew = euclidean_edges(g["nodes"], 8)
    wf = WarpField(EDGraph(g["nodes"], e, ew, node_coverage=cov), vol)
    wf.set_node_transforms(g["R"], g["T"])
    packed = wf.packed_nodes()
    for normals in (False, True):
        ref = torch.empty_like(pts)
        vv = v1.to(torch.uint8)
        call("ofx_deform_points", ptr(pts), pts.shape[0], ptr(a1), ptr(w1), ptr(vv), 4, ptr(packed), packed.shape[0],
             1 if normals else 0, ptr(ref), stream_ptr())
        out = torch.ops.ofx.deform_points(pts, a1, w1, v1, packed, normals)
        assert torch.equal(ref, out)


def test_opcheck_skin_and_deform(cuda, small):
    nodes = torch.from_numpy(small["nodes"]).to(cuda)
    pts = nodes[:200] + 0.01
    torch.library.opcheck(torch.ops.ofx.skin_points.default, (pts, nodes, float(small["node_coverage"]), 4))
    a, w, v = torch.ops.ofx.skin_points(pts, nodes, float(small["node_coverage"]), 4)
    packed = torch.zeros((nodes.shape[0], 16), device=cuda)
    packed[:, 0] = 1.0
    torch.library.opcheck(torch.ops.ofx.deform_points.default, (pts, a, w, v, packed, False))


def test_integrate_op_equals_direct_call(cuda, small):
    """The whole two-frame fusion of the golden volume through torch.ops.ofx.integrate (the shim) and through
    the raw ofx_integrate / ofx_integrate_palette calls: identical tsdf / weight / colour / update counts."""
    from types import SimpleNamespace
    from occlusionfusion_amd import EDGraph, WarpField, TSDFVolume
    from occlusionfusion_amd.synthetic import euclidean_edges
    g = small
    vols = []
    for direct in (False, True):
        fopt = SimpleNamespace(source_frame=0, skip_rate=1)
        vol = TSDFVolume.from_grid(g["origin"], float(g["voxel_size"]), g["dims"], tuple(g["intr"]), fopt, device=cuda)
        e, ew = euclidean_edges(g["nodes"], 8)
        wf = WarpField(EDGraph(g["nodes"], e, ew, node_coverage=float(g["node_coverage"])), vol)
        for fr, im in ((0, g["im0"]), (1, g["im1"])):
            if fr == 1:
                wf.frame_id = 1
                wf.set_node_transforms(g["R"], g["T"])
            vol.update(im, fr)
            if not direct:
                vol.integrate_device(count_updates=True)
                continue
            cam = vol.camera()
            if fr == 0:
                call("ofx_integrate", byref(vol.desc), byref(cam), ptr(vol.depth_t), ptr(vol.color_t), 0, None, 0, 1,
                     None, 0, None, None, 1.0, ptr(vol.tsdf_b), ptr(vol.weight_b), ptr(vol.color_b),
                     ptr(vol.n_updated), stream_ptr())
            else:
                c = wf.skin_tsdf_cache()
                call("ofx_integrate_palette", byref(vol.desc), byref(cam), ptr(vol.depth_t), ptr(vol.color_t),
                     ptr(wf.packed_nodes()), wf.num_nodes, c.k, ptr(c.brick_list), c.n_list, ptr(c.anchors),
                     ptr(c.weights), ptr(c.pal_ids), ptr(c.pal_n), ptr(c.local), 1.0, ptr(vol.tsdf_b),
                     ptr(vol.weight_b), ptr(vol.color_b), ptr(vol.n_updated), stream_ptr())
        vols.append(vol)
    a, b = vols
    for x, y in ((a.tsdf_b, b.tsdf_b), (a.weight_b, b.weight_b), (a.color_b, b.color_b), (a.n_updated, b.n_updated)):
        assert torch.equal(x, y)
    t1 = a.get_volume()[0]
    assert np.array_equal(t1, g["tsdf1"].reshape(tuple(g["dims"])))


def test_gn_solve_op_equals_direct_call(cuda, golden_dir):
    from occlusionfusion_amd import GaussNewtonSolver
    g = np.load(os.path.join(golden_dir, "gn_small.npz"), allow_pickle=False)
    inputs = (g["nodes"], g["edges"], g["edge_weights"], g["tpos"], g["conf"], g["src"], g["anchors"], g["weights"],
              g["tgt"], g["intr"])
    via_op = GaussNewtonSolver(len(g["nodes"]), 1000).optimize(*inputs)
    s = GaussNewtonSolver(len(g["nodes"]), 1000)
    args, N, M = s._problem(*inputs, None, None, None, None)
    pb = _lib.GnProblem()
    pb.n_nodes, pb.n_matches, pb.n_neighbors = N, M, args[1].shape[1]
    (pb.nodes, pb.edges, pb.edge_weights, pb.target_node_pos, pb.node_conf, pb.src, pb.anchors, pb.weights,
     pb.tgt) = (ptr(t) for t in args[:9])
    pb.target_px = pb.target_py = pb.prev_rot = pb.prev_trans = None
    pb.fx, pb.fy, pb.cx, pb.cy = args[13]
    p = _lib.GnParams()
    fp, ip = s._plist()
    (p.lambda_flow, p.lambda_depth, p.lambda_arap, p.lambda_motion, p.lm_factor, p.stop_loss_diff, p.pcg_tol,
     p.pcg_err_tol, p.precond_rot_tol) = fp
    p.num_iter, p.use_edge_weighting, p.pcg_max_iter, p.pcg_warm, p.mode, p.precond_every, p.precond = ip
    rot, trans = torch.empty((N, 3, 3), device=cuda), torch.empty((N, 3), device=cuda)
    status, loss = torch.zeros(5, dtype=torch.int32, device=cuda), torch.zeros((ip[0], 4), dtype=torch.float64,
                                                                                device=cuda)
    r = _lib.GnResult()
    r.rot, r.trans, r.status, r.loss_log = ptr(rot), ptr(trans), ptr(status), ptr(loss)
    call("ofx_gn_solve", s._h, byref(pb), byref(p), byref(r), stream_ptr())
    assert torch.equal(rot, via_op["node_rotations"]) and torch.equal(trans, via_op["node_translations"])
    assert torch.equal(status, via_op["_status"]) and torch.equal(loss, via_op["_loss"])


def test_ops_run_on_the_current_stream(cuda, small):
    """Work enqueued by an operator on a side stream is ordered on that stream (the current-stream convention)."""
    nodes = torch.from_numpy(small["nodes"]).to(cuda)
    pts = (nodes.repeat(200, 1) + 0.001).contiguous()
    side = torch.cuda.Stream(cuda)
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
        a, w, v = torch.ops.ofx.skin_points(pts, nodes, float(small["node_coverage"]), 4)
        ev = torch.cuda.Event()
        ev.record(side)
    ev.synchronize()
    a0, w0, v0 = torch.ops.ofx.skin_points(pts, nodes, float(small["node_coverage"]), 4)
    assert torch.equal(a, a0) and torch.equal(w, w0)
