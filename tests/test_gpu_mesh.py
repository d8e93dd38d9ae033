"""GPU parity of surface extraction: compute_truncated_region (tsdf.py:704-745),
masked / unmasked marching cubes (tsdf.py:755,794) and the get_mesh / get_point_cloud colours
(tsdf.py:757-767,796-807) through the C ABI vs the oracle restatement: bit-exact masks, vertex
positions / normals / values (matched by edge key), identical faces, identical colours."""
import os
from collections import Counter

import numpy as np
import pytest
import torch

from oracle import fusion_oracle as fo

pytestmark = pytest.mark.gpu


class _Opt:
    source_frame = 0
    skip_rate = 1


def _fused_small(golden_dir):
    from occlusionfusion_amd import TSDFVolume, EDGraph, WarpField
    from occlusionfusion_amd.synthetic import euclidean_edges
    g = np.load(os.path.join(golden_dir, "integrate_small.npz"), allow_pickle=False)
    vol = TSDFVolume.from_grid(g["origin"], float(g["voxel_size"]), g["dims"], tuple(g["intr"]), _Opt())
    vol.integrate({"im": g["im0"], "id": 0})
    e, w = euclidean_edges(g["nodes"], 8)
    wf = WarpField(EDGraph(g["nodes"], e, w, node_coverage=float(g["node_coverage"])), vol)
    wf.frame_id = 1
    wf.set_node_transforms(g["R"], g["T"])
    vol.integrate({"im": g["im1"], "id": 1})
    return vol, g


def _volume_from(arr, color=None):
    from occlusionfusion_amd import TSDFVolume, _lib
    vol = TSDFVolume.from_grid(np.array([-0.1, 0.2, 0.7], np.float32), 0.004, arr.shape, (100.0, 100.0, 50.0, 40.0), _Opt())
    for a, dst in ((arr, vol.tsdf_b), (color, vol.color_b)):
        if a is None:
            continue
        src = torch.from_numpy(np.ascontiguousarray(a, np.float32)).to(vol.device)
        _lib.call("ofx_volume_from_dense", _lib.byref(vol.desc), _lib.ptr(src), _lib.ptr(dst), _lib.stream_ptr())
    return vol


def _check_mesh(m, ref):
    verts, faces, normals, values, keys = ref
    k = m["keys"].cpu().numpy()
    order = np.argsort(k)
    np.testing.assert_array_equal(k[order], keys)
    np.testing.assert_array_equal(m["verts"].cpu().numpy()[order], verts)
    np.testing.assert_array_equal(m["normals"].cpu().numpy()[order], normals)
    np.testing.assert_array_equal(m["values"].cpu().numpy()[order], values)
    fk = k[m["faces"].cpu().numpy().astype(np.int64)]
    rk = keys[faces]
    assert sorted(map(tuple, fk)) == sorted(map(tuple, rk))


def test_truncated_region_bitexact(cuda, golden_dir):
    from occlusionfusion_amd import TSDFVolume
    vol, g = _fused_small(golden_dir)
    t, c, w = vol.get_volume()
    ref = fo.compute_truncated_region(t, 1.2)
    np.testing.assert_array_equal(TSDFVolume.compute_truncated_region(t, 1.2), ref)
    assert ref.sum() > 1000
    rng = np.random.default_rng(0)
    r = rng.uniform(-1.5, 1.5, (19, 23, 17)).astype(np.float32)
    r[3, 4, 5] = np.nan
    for md in (0.3, 1.2):
        np.testing.assert_array_equal(TSDFVolume.compute_truncated_region(r, md), fo.compute_truncated_region(r, md))


def test_masked_marching_cubes_and_get_mesh_bitexact(cuda, golden_dir):
    vol, g = _fused_small(golden_dir)
    t, c, w = vol.get_volume()
    m = vol.extract_mesh_device(use_mask=True, with_values=True, with_keys=True)
    ref = fo.marching_cubes(t, 0.0, fo.compute_truncated_region(t, 1.2))
    assert len(ref[0]) > 500
    _check_mesh(m, ref)
    verts, faces, norms, colors = vol.get_mesh()
    rv, rf, rn, rc = fo.get_mesh(t, c, vol._voxel_size, vol._vol_origin)
    k = m["keys"].cpu().numpy()
    order = np.argsort(k)
    np.testing.assert_array_equal(verts[order], rv)
    np.testing.assert_array_equal(norms[order], rn)
    np.testing.assert_array_equal(colors[order], rc)
    assert colors.dtype == np.uint8 and faces.shape[1] == 3 and len(faces) == len(rf)


def test_unmasked_sphere_point_cloud_closed_surface(cuda):
    X = np.arange(40)[:, None, None]
    Y = np.arange(36)[None, :, None]
    Z = np.arange(45)[None, None, :]
    sdf = (np.sqrt((X - 19.3) ** 2 + (Y - 17.6) ** 2 + (Z - 22.1) ** 2) - 11.4).astype(np.float32)
    col = ((X * 3 % 256) * 65536 + (Y * 5 % 256) * 256 + (Z * 7 % 256) + 0 * sdf).astype(np.float32)
    vol = _volume_from(sdf, col)
    m = vol.extract_mesh_device(use_mask=False, with_values=True, with_keys=True)
    ref = fo.marching_cubes(sdf, 0.0, None)
    _check_mesh(m, ref)
    f = m["faces"].cpu().numpy()
    de = Counter()
    for a, b, cc in f:
        de[(a, b)] += 1; de[(b, cc)] += 1; de[(cc, a)] += 1
    assert all(n == 1 for n in de.values()) and all((b, a) in de for (a, b) in de)   # closed, consistently wound
    v = m["verts"].cpu().numpy()
    fn = np.cross(v[f[:, 1]] - v[f[:, 0]], v[f[:, 2]] - v[f[:, 0]])
    assert (np.einsum("ij,ij->i", fn, m["normals"].cpu().numpy()[f[:, 0]]) > 0).all()   # outward
    pc = vol.get_point_cloud()
    order = np.argsort(m["keys"].cpu().numpy())
    world = ref[0] * np.float32(vol._voxel_size) + vol._vol_origin
    np.testing.assert_array_equal(pc[order, :3], world)
    np.testing.assert_array_equal(pc[order, 3:].astype(np.uint8), fo.mesh_colors(ref[0], col))


def _shards_of(full, world):
    """Slab shards holding the full volume's bricks (the bricked layout is x-column-major: a slice)."""
    from occlusionfusion_amd import TSDFVolume
    out = []
    c = full.brick_column_slots()
    for r in range(world):
        sh = TSDFVolume.from_grid(full._vol_origin, full._voxel_size, full._vol_dim,
                                  (full.cam_intr[0, 0], full.cam_intr[1, 1], full.cam_intr[0, 2], full.cam_intr[1, 2]),
                                  _Opt(), shard=(r, world))
        sh.tsdf_b.copy_(full.tsdf_b[c * sh.brick_x0: c * sh.brick_x1])
        sh.color_b.copy_(full.color_b[c * sh.brick_x0: c * sh.brick_x1])
        out.append(sh)
    return out


def _sharded_mesh(shards, **kw):
    from occlusionfusion_amd.sharding import merge_shard_meshes
    parts = []
    for r, sh in enumerate(shards):
        lo = shards[r - 1].boundary_columns()[1] if r > 0 else None
        hi = shards[r + 1].boundary_columns()[0] if r < len(shards) - 1 else None
        parts.append(sh.extract_mesh_shard(lo, hi, with_values=True, **kw))
    return merge_shard_meshes(parts, shards[0]._vol_dim), parts


def _assert_same_mesh(merged, full, use_mask):
    m = full.extract_mesh_device(use_mask=use_mask, with_values=True, with_keys=True)
    world, colors = full._mesh_world_colors(m["verts"])
    for name, ref in (("verts", m["verts"]), ("faces", m["faces"]), ("normals", m["normals"]),
                      ("values", m["values"]), ("keys", m["keys"]), ("world", world), ("colors", colors)):
        assert torch.equal(merged[name], ref), name
    return m


@pytest.mark.parametrize("world", [1, 2, 3])
def test_sharded_marching_cubes_equals_whole_volume(cuda, golden_dir, world):
    """Slab-sharded get_mesh (halo of one brick column per neighbour, each shard meshing
    the cells whose far corner lies in its slab, key merge) == the whole volume's, bit for bit: vertices,
    vertex order, faces, normals, values, world coordinates and colours."""
    vol, g = _fused_small(golden_dir)
    merged, parts = _sharded_mesh(_shards_of(vol, world), use_mask=True, max_diff=1.2)
    m = _assert_same_mesh(merged, vol, True)
    assert m["faces"].shape[0] > 500
    if world > 1:   # vertices on the slab boundaries are shared by two parts
        assert sum(p["keys"].shape[0] for p in parts) > m["keys"].shape[0]


@pytest.mark.parametrize("world", [2, 5])
def test_sharded_point_cloud_sphere_across_slabs(cuda, world):
    """Unmasked marching cubes of a sphere cut by every slab boundary (5 shards of 40 voxels: one brick
    column each) == the whole volume's."""
    X = np.arange(40)[:, None, None]
    Y = np.arange(36)[None, :, None]
    Z = np.arange(45)[None, None, :]
    sdf = (np.sqrt((X - 19.3) ** 2 + (Y - 17.6) ** 2 + (Z - 22.1) ** 2) - 15.4).astype(np.float32)
    col = ((X * 3 % 256) * 65536 + (Y * 5 % 256) * 256 + (Z * 7 % 256) + 0 * sdf).astype(np.float32)
    vol = _volume_from(sdf, col)
    merged, _ = _sharded_mesh(_shards_of(vol, world), use_mask=False)
    _assert_same_mesh(merged, vol, False)


def test_mesh_shard_halo_arguments(cuda):
    from occlusionfusion_amd import TSDFVolume
    sh = TSDFVolume.from_grid(np.zeros(3, np.float32), 0.01, (32, 8, 8), (1.0, 1.0, 0.0, 0.0), _Opt(), shard=(1, 3))
    with pytest.raises(ValueError):
        sh.extract_mesh_shard()                      # a middle shard needs both halo columns
    c = sh.brick_column_slots()
    with pytest.raises(ValueError):
        sh.extract_mesh_shard(torch.zeros((2, c - 1), device=sh.device), torch.zeros((2, c), device=sh.device))


def test_mesh_empty_and_sharded_refused(cuda):
    from occlusionfusion_amd import TSDFVolume, _lib
    vol = _volume_from(np.ones((10, 12, 9), np.float32))
    m = vol.extract_mesh_device(use_mask=True)
    assert m["verts"].shape[0] == 0 and m["faces"].shape[0] == 0
    sh = TSDFVolume.from_grid(np.zeros(3, np.float32), 0.01, (32, 8, 8), (1.0, 1.0, 0.0, 0.0), _Opt(), shard=(0, 2))
    with pytest.raises(_lib.OfxError):
        sh.extract_mesh_device()
