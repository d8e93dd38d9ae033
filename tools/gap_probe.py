"""Tuning probe (not product): stream idle time at GN-step boundaries — from the event after a PCG chunk's last launch
(its drained launches included) to the event enqueued with the next GN step's first kernel — on the bench's config-3
sequence. Needs the stamps build (see tools/pcg_stamps.py):
    OFX_LIB=tools/bin/libofx_stamps.so python tools/gap_probe.py
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from occlusionfusion_amd import _lib  # noqa: E402
from occlusionfusion_amd import synthetic as S  # noqa: E402
from occlusionfusion_amd.pipeline import FusionPipeline  # noqa: E402

assert "stamps" in _lib.LIB_PATH, "run with OFX_LIB=tools/bin/libofx_stamps.so"
fn = _lib.lib.ofx_gn_gaps
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
fn.restype = ctypes.c_int32
dev = torch.device("cuda", 0)
cfg = S.BASELINE_CONFIGS[3]
seq = S.config_sequence(3, device=dev)
D = cfg["dims"]
pipe = FusionPipeline(seq, cfg["origin"], cfg["voxel"], (D, D, D), device=dev)
frames = [pipe.prepare(t) for t in range(34)]
pipe.integrate_source(frames[0])
for t in range(1, 4):
    pipe.step(frames[t], t, next_fi=frames[t + 1])
torch.cuda.synchronize()
ms, n = ctypes.c_double(), ctypes.c_int64()
for h in [s[0] for s in pipe.solver._slots]:
    fn(h, ctypes.byref(ms), ctypes.byref(n))
for t in range(4, 32):
    pipe.step(frames[t], t, next_fi=frames[t + 1])
pipe.solver.drain()
torch.cuda.synchronize()
tot, cnt = 0.0, 0
for h in [s[0] for s in pipe.solver._slots]:
    fn(h, ctypes.byref(ms), ctypes.byref(n))
    tot += ms.value
    cnt += n.value
print(f"GN-step boundary gaps: {cnt} over 28 frames (steps 1-9), {1e3 * tot / max(1, cnt):.2f} us each, {tot / 28:.3f} ms per frame")
