"""GPU: TSDF raycast (new capability — the reference renders no TSDF; parity unpinned against it) equals
its oracle restatement (oracle/fusion_oracle.py::raycast, f32 op for op) bit for bit, and sees the scene that
was fused: the raycast depth of a fused frame lies within a voxel of that frame's own depth."""
import os

import numpy as np
import pytest

from oracle import fusion_oracle as fo

pytestmark = pytest.mark.gpu


class _Opt:
    source_frame = 0
    skip_rate = 1


def _compare(vol, rows=None, z_near=0.1, z_far=10.0):
    t, c, w = vol.get_volume()
    H, W = (int(x) for x in vol.depth_t.shape)
    K = vol.cam_intr
    intr = (K[0, 0], K[1, 1], K[0, 2], K[1, 2])
    d, n, col = (x.cpu().numpy() for x in vol.raycast(z_near=z_near, z_far=z_far))
    od, on, oc = fo.raycast(t, w, c, vol._vol_origin, vol._voxel_size, intr, H, W, z_near, z_far, rows=rows)
    r = slice(None) if rows is None else rows
    np.testing.assert_array_equal(d[r], od[r])
    np.testing.assert_array_equal(n[r], on[r])
    np.testing.assert_array_equal(col[r], oc[r])
    return d


def test_raycast_golden_volume_bitexact(cuda, golden_dir):
    from occlusionfusion_amd import EDGraph, TSDFVolume, WarpField
    from occlusionfusion_amd.synthetic import euclidean_edges
    g = np.load(os.path.join(golden_dir, "integrate_small.npz"), allow_pickle=False)
    vol = TSDFVolume.from_grid(g["origin"], float(g["voxel_size"]), g["dims"], tuple(g["intr"]), _Opt(), device=cuda)
    vol.integrate({"im": g["im0"], "id": 0})
    d0 = _compare(vol)
    dep = g["im0"][5]
    m = (d0 > 0) & (dep > 0)
    assert m.sum() > 2000
    assert np.median(np.abs(d0[m] - dep[m])) < float(g["voxel_size"])
    e, w = euclidean_edges(g["nodes"], 8)
    wf = WarpField(EDGraph(g["nodes"], e, w, node_coverage=float(g["node_coverage"])), vol)
    wf.frame_id = 1
    wf.set_node_transforms(g["R"], g["T"])
    vol.integrate({"im": g["im1"], "id": 1})
    _compare(vol)
    _compare(vol, z_near=1.3, z_far=1.6)          # clipped range


@pytest.mark.parametrize("config", [1, 3])
def test_raycast_config_volume(cuda, config):
    from occlusionfusion_amd import synthetic as S
    from occlusionfusion_amd.pipeline import FusionPipeline
    c = S.BASELINE_CONFIGS[config]
    seq = S.config_sequence(config)
    D = c["dims"]
    pipe = FusionPipeline(seq, c["origin"], c["voxel"], (D, D, D), device=cuda)
    f0 = pipe.prepare(0)
    pipe.integrate_source(f0)
    H = seq.cam.height
    rows = np.arange(0, H, 8 if config == 3 else 1)
    d = _compare(pipe.vol, rows=rows)
    dep = f0.im[5].cpu().numpy()
    m = (d > 0) & (dep > 0)
    m[np.setdiff1d(np.arange(H), rows)] = False
    assert m.sum() > 1000
    assert np.median(np.abs(d[m] - dep[m])) < c["voxel"]


def test_raycast_axis_rays_and_inside_camera(cuda):
    """Edge cases of the slab test: integer principal point (the centre column / row has dx = 0 / dy = 0 exactly:
    the axis-parallel branch), a volume that contains the camera (entry clamped by z_near) and one that does not
    (rays whose box interval is empty)."""
    from types import SimpleNamespace
    from occlusionfusion_amd import TSDFVolume
    from occlusionfusion_amd import synthetic as S
    cam = S.Intrinsics(100.0, 100.0, 40.0, 30.0, 80, 60)
    depth = S.SphereScene(occluder=False).render(cam, 0, np.random.default_rng(0))
    im = S.make_image(depth)
    for origin in ((-0.6, -0.5, 0.9), (-0.6, -0.5, -0.2)):          # in front of / around the camera
        vol = TSDFVolume.from_grid(origin, 0.02, (64, 50, 60), (cam.fx, cam.fy, cam.cx, cam.cy),
                                   SimpleNamespace(source_frame=0, skip_rate=1), device=cuda)
        vol.integrate({"im": im, "id": 0})
        for zn, zf in ((0.1, 10.0), (1.2, 1.5), (0.05, 0.06)):
            d = _compare(vol, z_near=zn, z_far=zf)
            if (zn, zf) == (0.1, 10.0) and origin[2] > 0:
                assert (d > 0).sum() > 500
            if zf < 0.5:
                assert not (d > 0).any()



def test_raycast_entering_inside_the_negative_band_reports_no_entry_hit(cuda):
    """Rays that start (z_near) behind the fused front surface, inside its observed negative band, have no
    positive sample before their first one: no surface is reported at the entry plane (a spurious hit at z_near
    before the fix), and the result still equals the oracle bit for bit."""
    from types import SimpleNamespace
    from occlusionfusion_amd import TSDFVolume
    from occlusionfusion_amd import synthetic as S
    cam = S.Intrinsics(100.0, 100.0, 40.0, 30.0, 80, 60)
    depth = S.SphereScene(occluder=False).render(cam, 0, np.random.default_rng(0))
    vol = TSDFVolume.from_grid((-0.6, -0.5, 0.9), 0.01, (128, 100, 100), (cam.fx, cam.fy, cam.cx, cam.cy),
                               SimpleNamespace(source_frame=0, skip_rate=1), device=cuda)
    vol.integrate({"im": S.make_image(depth), "id": 0})
    full = _compare(vol)
    zc = float(full[30, 40])
    assert zc > 0
    zn = zc + 0.01                       # 1 cm behind the front surface: inside the 4 cm truncation band
    d = _compare(vol, z_near=zn, z_far=10.0)
    inside = np.abs(full - zc) < 0.004   # pixels whose surface lies (about) where the centre ray's does
    assert inside.sum() > 10
    assert not (d[inside] == np.float32(zn)).any()
    assert not ((d > 0) & (d <= np.float32(zn))).any()
