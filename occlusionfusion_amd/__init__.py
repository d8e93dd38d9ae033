"""occlusionfusion_amd — MI355X-native non-rigid TSDF fusion hot path (warp + integrate + GN solve).

Drop-in shims of remmel/OcclusionFusion's fusion core (TSDFVolume, WarpField, Registration /
DeformNet.optimize) over libofx.so: hand-written HIP kernels for gfx950 behind a C ABI
(include/ofx.h). There is no CPU fallback: touching any shim loads the built library and raises
ImportError if it is missing. (`synthetic` and `build` are plain-Python helpers and load nothing.)
"""
_EXPORTS = {
    "TSDFVolume": "tsdf", "volume_geometry": "tsdf", "shard_bricks": "sharding", "match_range": "sharding",
    "WarpField": "warpfield", "EDGraph": "warpfield",
    "GaussNewtonSolver": "registration", "Registration": "registration",
    "FusionPipeline": "pipeline",
    "backproject_depth": "image_proc", "compute_mesh_from_depth": "image_proc", "depth_2_pc": "image_proc",
}

__all__ = list(_EXPORTS)


def __getattr__(name):
    if name in _EXPORTS:
        import importlib
        mod = importlib.import_module(f".{_EXPORTS[name]}", __name__)
        return getattr(mod, name)
    raise AttributeError(name)
