"""ctypes wrapper of oracle/libcpu_ref.so (C/OpenMP restatement) — TEST INFRASTRUCTURE ONLY."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libcpu_ref.so")


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def _lib():
    if not os.path.exists(LIB):
        build()
    lib = ctypes.CDLL(LIB)
    f = lib.ofxref_integrate
    f.restype = ctypes.c_int64
    P = ctypes.c_void_p
    f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, P, ctypes.c_double, P, ctypes.c_int64, ctypes.c_int, P, P,
                  P, ctypes.c_int, P, P, P, P, P, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_float,
                  ctypes.c_float, ctypes.c_float, ctypes.c_double, ctypes.c_double, P, P, P]
    return f


_F = None


def set_threads(n):
    """OpenMP thread count of the C restatement (bench.py's single-thread leg)."""
    lib = ctypes.CDLL(LIB if os.path.exists(LIB) else build())
    lib.ofxref_set_threads.argtypes = [ctypes.c_int]
    lib.ofxref_set_threads(int(n))


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def integrate(dims, origin, voxel_size, vox, depth, color_im, intr, tsdf, weight, color, warp=False, anchors=None,
              weights=None, valid=None, R=None, T=None, nodes=None, trunc=0.04, obs_weight=1.0):
    """In-place integrate of voxel ids `vox` (C-order) into flat f32 tsdf/weight/color (full volume
    arrays). Skin arrays (anchors (n,K) i32, weights (n,K) f32, valid (n,) u8) are per listed voxel."""
    global _F
    if _F is None:
        _F = _lib()
    c = lambda a, dt: None if a is None else np.ascontiguousarray(a, dt)
    vox = c(vox, np.int64)
    origin = c(origin, np.float32)
    depth, color_im = c(depth, np.float32), c(color_im, np.float32)
    anchors, weights, valid = c(anchors, np.int32), c(weights, np.float32), c(valid, np.uint8)
    R, T, nodes = c(R, np.float32), c(T, np.float32), c(nodes, np.float32)
    K = 0 if anchors is None else anchors.shape[1]
    H, W = depth.shape
    fx, fy, cx, cy = (float(v) for v in intr)
    return _F(int(dims[0]), int(dims[1]), int(dims[2]), _p(origin), float(voxel_size), _p(vox), vox.size,
              1 if warp else 0, _p(anchors), _p(weights), _p(valid), K, _p(R), _p(T), _p(nodes), _p(depth),
              _p(color_im), W, H, fx, fy, cx, cy, float(trunc), float(obs_weight), _p(tsdf), _p(weight),
              _p(color))
