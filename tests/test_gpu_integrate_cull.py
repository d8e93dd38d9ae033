"""GPU: the per-frame brick cull in front of the warped palette integrate (ofx_integrate_palette_cull) is exact — the
volume after solver-driven warped frames is bit-identical with and without it, every brick it skips updates no voxel
(per-brick update counts equal), and it does skip bricks (on the synthetic scenes about half of the listed bricks update
nothing: the volume behind the surface and the occluded part). Its bound is conservative by construction (a box of
the palette nodes' rigid images of the brick, the skin weights' sum range, 1e-4 m and ±1 px margins); the
adversarial cases below push it: a volume that is mostly behind the camera / outside the image, and a pose that
moves the whole warped surface by a large translation."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _pipe(config, cuda):
    from occlusionfusion_amd import synthetic as S
    from occlusionfusion_amd.pipeline import FusionPipeline
    c = S.BASELINE_CONFIGS[config]
    seq = S.config_sequence(config, None, rank=0, device=cuda)
    D = c["dims"]
    pipe = FusionPipeline(seq, c["origin"], c["voxel"], (D, D, D), device=cuda)
    pipe.integrate_source(pipe.prepare(0))
    return pipe


def _twin_integrate(pipe, t, R=None, T=None):
    """Integrate frame t twice from the same state: with the cull and without; return both volumes, both per-brick
    update counts and the cull's flags."""
    vol = pipe.vol
    fi = pipe.prepare(t)
    if R is None:
        pipe.solve(fi)
        R, T = pipe.prev_rot, pipe.prev_trans
    keep = tuple(x.clone() for x in (vol.tsdf_b, vol.weight_b, vol.color_b))
    out = []
    for cull in (False, True):   # the culled run last: the volume keeps its (identical) result
        vol.tsdf_b, vol.weight_b, vol.color_b = (x.clone() for x in keep)
        vol.brick_cull = cull
        pipe.wf.set_node_transforms(R, T)
        pipe.wf.frame_id = t
        vol.frame_id = t - 1
        vol.update(fi.im, t)
        vol.n_updated.zero_()
        vol.integrate_device(count_updates=True)
        torch.cuda.synchronize()
        out.append((vol.tsdf_b.clone(), vol.weight_b.clone(), vol.color_b.clone(), vol.n_updated.clone()))
    n = pipe.wf.skin_tsdf_cache().n_list
    return out[::-1], vol._cull[1][:n].clone(), n


def _check(out, active, n):
    (t1, w1, c1, u1), (t0, w0, c0, u0) = out
    assert torch.equal(t1, t0) and torch.equal(w1, w0) and torch.equal(c1, c0)
    assert torch.equal(u1[:n], u0[:n])
    skipped = active == 0
    assert int(u0[:n][skipped].sum().item()) == 0          # a skipped brick would have updated nothing
    return int(skipped.sum().item())


def test_cull_is_exact_and_skips_bricks_config1(cuda):
    pipe = _pipe(1, cuda)
    for t in (1, 2):
        out, active, n = _twin_integrate(pipe, t)
        skipped = _check(out, active, n)
        assert skipped > 0.1 * n, (skipped, n)   # (the volume now holds frame t: the next frame fuses onto it)


def test_cull_is_exact_config3(cuda):
    pipe = _pipe(3, cuda)
    out, active, n = _twin_integrate(pipe, 1)
    skipped = _check(out, active, n)
    assert skipped > 0.2 * n, (skipped, n)


def test_cull_exact_under_large_motion(cuda):
    """Node transforms far from the solve's: a large common translation (most of the warped volume leaves the image
    or goes behind the camera) and a rotation of the whole graph about the camera axis."""
    pipe = _pipe(1, cuda)
    N = pipe.seq.nodes.shape[0]
    eye = torch.eye(3, device=cuda).repeat(N, 1, 1)
    for dt in ((0.0, 0.0, -0.9), (0.25, -0.1, 0.05), (0.0, 0.0, 0.3)):
        T = torch.tensor(dt, device=cuda).repeat(N, 1)
        out, active, n = _twin_integrate(pipe, 1, eye, T)
        _check(out, active, n)
    a = 0.6
    Rz = torch.tensor([[np.cos(a), -np.sin(a), 0.0], [np.sin(a), np.cos(a), 0.0], [0.0, 0.0, 1.0]], device=cuda,
                      dtype=torch.float32)
    g = torch.from_numpy(pipe.seq.nodes).to(cuda)
    T = (g @ Rz.T) - g          # node-relative form of a rigid rotation about the camera origin
    out, active, n = _twin_integrate(pipe, 1, Rz.repeat(N, 1, 1), T)
    _check(out, active, n)
