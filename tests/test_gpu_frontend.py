"""GPU parity of the correspondence front-end through the C ABI:
backproject_depth (csrc image_proc.cpp:351-401), compute_mesh_from_depth (image_proc.cpp:405-545) and the
Registration.optimize target cloud (geometry.py:44-59, registration_fusion.py:104-109,388-395).

Pinned by tests/golden/frontend_csrc.npz, which holds the REFERENCE C++'s own outputs (compiled from
/root/reference by oracle/build_ref.py) — bit-exact, including thresholds that tie with edge lengths. At
the full 640x448 frame size the mesh is checked through size-independent properties that fix it exactly:
the valid-triangle set (vectorised restatement), sequential first-use vertex numbering, vertex positions."""
import os

import numpy as np
import pytest
import torch

from oracle import fusion_oracle as fo

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def g(golden_dir):
    return np.load(os.path.join(golden_dir, "frontend_csrc.npz"), allow_pickle=False)


def test_backproject_float_and_ushort_bit_exact(g, cuda):
    from occlusionfusion_amd.image_proc import backproject_depth, backproject_depth_device
    fx, fy, cx, cy = [float(v) for v in g["intr"]]
    assert np.array_equal(backproject_depth(g["depth"], fx, fy, cx, cy), g["backproject_float"])
    assert np.array_equal(backproject_depth(g["depth_u16"], fx, fy, cx, cy, 1000.0), g["backproject_ushort"])
    # untouched where depth <= 0 (the C++ writes only valid pixels)
    d = torch.from_numpy(g["depth"]).to(cuda)
    out = torch.full((3,) + tuple(d.shape), 7.0, device=cuda)
    backproject_depth_device(d, fx, fy, cx, cy, out=out)
    o = out.cpu().numpy()
    inv = g["depth"] <= 0
    assert inv.any() and np.all(o[:, inv] == 7.0)
    assert np.array_equal(o[:, ~inv], g["backproject_float"][:, ~inv])


def test_depth_mesh_matches_reference_csrc(g, cuda):
    from occlusionfusion_amd.image_proc import compute_mesh_from_depth_device
    p = torch.from_numpy(g["backproject_float"]).to(cuda)
    for i, t in enumerate(g["thresholds"]):
        m = compute_mesh_from_depth_device(p, float(t))
        assert np.array_equal(m["vertices"].cpu().numpy(), g[f"mesh{i}_vertices"]), i
        assert np.array_equal(m["vertex_pixels"].cpu().numpy(), g[f"mesh{i}_pixels"]), i
        assert np.array_equal(m["faces"].cpu().numpy(), g[f"mesh{i}_faces"]), i


def test_depth_mesh_inplace_api(g, cuda):
    from occlusionfusion_amd.image_proc import compute_mesh_from_depth
    v, px, f = np.zeros((0,), np.float32), np.zeros((0,), np.int32), np.zeros((0,), np.int32)
    compute_mesh_from_depth(g["backproject_float"], float(g["thresholds"][0]), v, px, f)
    assert np.array_equal(v, g["mesh0_vertices"]) and np.array_equal(px, g["mesh0_pixels"])
    assert np.array_equal(f, g["mesh0_faces"])
    # no valid triangle: outputs stay zero-size (image_proc.cpp:520)
    v2, px2, f2 = np.zeros((0,), np.float32), np.zeros((0,), np.int32), np.zeros((0,), np.int32)
    assert compute_mesh_from_depth(np.zeros((3, 5, 4), np.float32), 0.05, v2, px2, f2) == (0, 0)
    assert v2.size == 0 and px2.size == 0 and f2.size == 0


def _valid_triangles(P, md):
    """vectorised restatement of the two triangle tests of image_proc.cpp:445-505 (Eigen's x0 + (x1 + x2))."""
    f32 = np.float32
    o00, o01, o10, o11 = P[:, :-1, :-1], P[:, 1:, :-1], P[:, :-1, 1:], P[:, 1:, 1:]

    def L(a, b):
        d = (a - b).astype(f32)
        s = d * d
        return np.sqrt((s[0] + (s[1] + s[2])).astype(f32))

    A = (o00[2] > 0) & (o01[2] > 0) & (o10[2] > 0) & (L(o00, o01) <= md) & (L(o00, o10) <= md) & (L(o01, o10) <= md)
    B = (o01[2] > 0) & (o10[2] > 0) & (o11[2] > 0) & (L(o10, o01) <= md) & (L(o10, o11) <= md) & (L(o01, o11) <= md)
    return A, B


def test_depth_mesh_full_frame_properties(cuda):
    from occlusionfusion_amd import synthetic as S
    from occlusionfusion_amd.image_proc import backproject_depth_device, compute_mesh_from_depth_device
    cam = S.Intrinsics(525.0, 525.0, 319.5, 239.5 - 16, 640, 448)
    d = S.SphereScene().render(cam, 2, np.random.default_rng(7)).astype(np.float32)
    P = backproject_depth_device(torch.from_numpy(d).to(cuda), cam.fx, cam.fy, cam.cx, cam.cy)
    md = np.float32(0.05)
    m = compute_mesh_from_depth_device(P, float(md))
    V, F = m["vertices"].cpu().numpy(), m["faces"].cpu().numpy()
    px = m["vertex_pixels"].cpu().numpy()
    Pn = P.cpu().numpy()
    A, B = _valid_triangles(Pn, md)
    H, W = d.shape
    # faces: exactly the valid triangles, quads row-major, A before B, with the C++ vertex order
    q = np.stack([A, B], -1).reshape(-1)
    t = np.nonzero(q)[0]
    assert F.shape[0] == t.size > 100000
    qy, qx, tri = t // 2 // (W - 1), t // 2 % (W - 1), t % 2
    corner = {0: [(0, 0), (0, 1), (1, 0)], 1: [(1, 1), (1, 0), (0, 1)]}   # (dx, dy) of (x, y)
    for c in range(3):
        dx = np.where(tri == 0, [a[0] for a in corner[0]][c], [a[0] for a in corner[1]][c])
        dy = np.where(tri == 0, [a[1] for a in corner[0]][c], [a[1] for a in corner[1]][c])
        assert np.array_equal(px[F[:, c], 0], qx + dx) and np.array_equal(px[F[:, c], 1], qy + dy)
    # vertices numbered on first use: first occurrences in the flattened face list are 0, 1, 2, ...
    flat = F.reshape(-1)
    _, first = np.unique(flat, return_index=True)
    assert np.array_equal(flat[np.sort(first)], np.arange(V.shape[0]))
    # positions are the point image at the vertex pixels
    assert np.array_equal(V, Pn[:, px[:, 1], px[:, 0]].T)


def test_depth_mesh_edge_cases(cuda):
    from occlusionfusion_amd import _lib
    from occlusionfusion_amd.image_proc import compute_mesh_from_depth_device
    p = torch.zeros((3, 2, 2), device=cuda)
    p[2] = 1.0
    m = compute_mesh_from_depth_device(p, 0.05)        # one quad, 2 triangles of zero-length edges
    assert m["faces"].cpu().numpy().tolist() == [[0, 1, 2], [3, 2, 1]]
    assert m["vertex_pixels"].cpu().numpy().tolist() == [[0, 0], [0, 1], [1, 0], [1, 1]]
    with pytest.raises(_lib.OfxError):
        compute_mesh_from_depth_device(torch.ones((3, 1, 8), device=cuda), 0.05)


def test_target_point_cloud_bit_exact(g, cuda):
    from occlusionfusion_amd.image_proc import depth_2_pc_device
    pts, pmap = depth_2_pc_device(torch.from_numpy(g["depth"]).to(cuda), g["K"])
    assert np.array_equal(pts.cpu().numpy(), g["target_pc"])
    assert np.array_equal(pmap.cpu().numpy(), g["target_pix_map"])
    # full frame against the oracle; empty depth -> empty cloud, all -1
    from occlusionfusion_amd import synthetic as S
    cam = S.Intrinsics(525.0, 525.0, 319.5, 239.5 - 16, 640, 448)
    d = S.SphereScene().render(cam, 3, np.random.default_rng(9)).astype(np.float32)
    K = np.array([[cam.fx, 0, cam.cx], [0, cam.fy, cam.cy], [0, 0, 1]], np.float64)
    pc, pm = fo.target_point_cloud(d, K)
    pts, pmap = depth_2_pc_device(torch.from_numpy(d).to(cuda), K)
    assert np.array_equal(pts.cpu().numpy(), pc) and np.array_equal(pmap.cpu().numpy(), pm)
    pts, pmap = depth_2_pc_device(torch.zeros((48, 64), device=cuda), K)
    assert pts.shape == (0, 3) and bool((pmap == -1).all())
