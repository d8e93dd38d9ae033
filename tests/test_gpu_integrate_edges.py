"""GPU: the certified fast arithmetic of the integrate kernels (f32 pixel rounding with an f64 fallback near
ties, cheap SDF rounding certificate) against the numpy oracle on ADVERSARIAL points, bit for bit:
projections within 1e-12 .. 3e-4 px of a half-integer rounding tie, the image border (-0.5, W-0.5, the
-0 -> 0 case), subnormal / tiny / zero / negative / non-finite depths, and random old tsdf / weight / colour
with depths around the truncation band. Runs through ofx_integrate_points (TSDFVolume.integrate_points)."""
import numpy as np
import pytest
import torch

from oracle import fusion_oracle as fo

pytestmark = pytest.mark.gpu

F32 = np.float32


def adversarial_points(cam, n, rng):
    fx, fy, cx, cy = (F32(v) for v in (cam.fx, cam.fy, cam.cx, cam.cy))
    z = rng.uniform(0.3, 3.5, n).astype(F32)
    # target pixel coordinates: a half-integer tie + a tiny offset, or the image borders
    offs = np.array([0, 1e-12, -1e-12, 1e-9, -1e-9, 1e-7, -1e-7, 1e-6, -1e-6, 1e-5, -1e-5, 1e-4, -1e-4, 3e-4, -3e-4,
                     0.25, 0.5])
    su = rng.integers(-2, cam.width + 2, n) + 0.5 + rng.choice(offs, n)
    sv = rng.integers(-2, cam.height + 2, n) + 0.5 + rng.choice(offs, n)
    border = rng.random(n) < 0.1
    su[border] = rng.choice([-0.5, -0.4999999, -0.5000001, cam.width - 0.5, cam.width - 0.5000001], border.sum())
    x = ((su - cx) * z.astype(np.float64) / fx).astype(F32)
    y = ((sv - cy) * z.astype(np.float64) / fy).astype(F32)
    pts = np.stack([x, y, z], 1)
    # degenerate depths
    m = rng.random(n) < 0.02
    pts[m, 2] = rng.choice(np.array([0.0, -0.0, -1.0, 1e-40, 1e-38, 1e-31, 1e-29, np.inf, np.nan], F32), m.sum())
    m = rng.random(n) < 0.005
    pts[m, 0] = 0.0
    pts[m, 2] = np.array(1e-40, F32)
    return pts


def test_integrate_points_adversarial_bitexact(cuda, tmp_path):
    from types import SimpleNamespace
    from occlusionfusion_amd import TSDFVolume
    from occlusionfusion_amd import synthetic as S
    rng = np.random.default_rng(7)
    cam = S.bench_camera()
    D = (48, 64, 40)
    V = int(np.prod(D))
    n = V
    pts = adversarial_points(cam, n, rng)
    vox = rng.permutation(V).astype(np.int64)
    valid = rng.random(n) < 0.97
    # depth around each point's z (inside / at / beyond the truncation band) at its pixel; random elsewhere
    depth = rng.uniform(0.2, 3.6, (cam.height, cam.width)).astype(F32)
    depth[rng.random(depth.shape) < 0.05] = 0.0
    zz = pts[:, 2].astype(np.float64)
    with np.errstate(all="ignore"):
        u = np.rint(pts[:, 0].astype(np.float64) * np.float64(F32(cam.fx)) / zz + np.float64(F32(cam.cx)))
        v = np.rint(pts[:, 1].astype(np.float64) * np.float64(F32(cam.fy)) / zz + np.float64(F32(cam.cy)))
    ok = np.isfinite(u) & np.isfinite(v) & (u >= 0) & (u < cam.width) & (v >= 0) & (v < cam.height) & (zz > 0)
    sel = np.nonzero(ok)[0][::3]
    depth[v[sel].astype(int), u[sel].astype(int)] = (zz[sel] + rng.choice([-0.05, -0.04, -0.0399999, 0.0, 0.01, 0.04,
                                                                          0.3], sel.size)).astype(F32)
    im = S.make_image(depth)
    # random old state
    t0 = rng.uniform(-1, 1, V).astype(F32)
    w0 = rng.choice(np.array([0, 1, 2, 3, 7, 0.5, 1.25], F32), V)
    c0 = np.floor(rng.uniform(0, 2 ** 24 - 1, V)).astype(F32)
    np.save(tmp_path / "vol.npy", np.stack([t0.reshape(D), c0.reshape(D), w0.reshape(D)]))
    fopt = SimpleNamespace(source_frame=0, skip_rate=1)
    intr = (cam.fx, cam.fy, cam.cx, cam.cy)
    vol = TSDFVolume.from_grid((-0.5, -0.5, 0.5), 0.01, D, intr, fopt, device=cuda)
    vol.load_volume(str(tmp_path / "vol.npy"))
    vol.update(im, 3)
    cnt = vol.integrate_points(pts, vox, valid, obs_weight=1.0, count_updates=True)
    t_gpu, c_gpu, w_gpu = (a.reshape(-1) for a in vol.get_volume())
    # oracle on the same points, in voxel order
    t, w, c = t0.copy(), w0.copy(), c0.copy()
    P = np.zeros((V, 3), F32)
    P[vox] = pts
    vm = np.zeros(V, bool)
    vm[vox] = valid
    with np.errstate(all="ignore"):
        n_upd = fo.integrate(t, w, c, P, vm, fo.depth_of(im), fo.pack_color(im), intr)
    assert n_upd > V // 20
    assert int(cnt.item()) == n_upd
    np.testing.assert_array_equal(w_gpu, w)
    np.testing.assert_array_equal(t_gpu, t)
    np.testing.assert_array_equal(c_gpu, c)
