"""Tuning study (not product): per-phase clock stamps of the persistent PCG (k_pcg_persist) on the bench workload.

Needs the stamps build (built on the box: python -c "from occlusionfusion_amd import build;
build.build(out='scratch/libofx_stamps.so', defines=['OFX_STAMPS'])"), then
OFX_PCG_PERSIST=1 OFX_LIB=scratch/libofx_stamps.so python tools/persist_stamps.py
Stamps (s_memtime cycles) per iteration and workgroup: 0 start | 1 m gathered (compute wave 0) | 2 SpMV done |
3 partials polled (poll wave) | 4 after the scalar barrier | 5 m published + wave sums | 6 after the partial barrier |
7 workgroup partials published (poll wave).
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from occlusionfusion_amd import _lib
from occlusionfusion_amd import synthetic as S
from occlusionfusion_amd.pipeline import FusionPipeline

assert "stamps" in _lib.LIB_PATH, "run with OFX_LIB=<stamps build>"
os.environ.setdefault("OFX_PCG_PERSIST", "1")
fn = _lib.lib.ofx_gn_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
fn.restype = ctypes.c_int32
dev = torch.device("cuda", 0)
seq = S.config_sequence(3, device=dev)
D = int(os.environ.get("DIMS", "128"))
pipe = FusionPipeline(seq, (-D * 0.002, -D * 0.002, 0.5), 0.004, (D, D, D), device=dev)
frames = [pipe.prepare(t) for t in range(8)]
pipe.integrate_source(frames[0])
for t in range(1, 6):
    pipe.step(frames[t], t)
torch.cuda.synchronize()
h = pipe.solver._h
print("pcg form", pipe.solver.pcg_form())
fn(h, None, 0)                      # allocate + clear
pipe.step(frames[6], 6)             # stamps of the LAST GN step's solve remain (each solve overwrites)
torch.cuda.synchronize()
nw = pipe.solver.info()[4] // 8
buf = np.zeros(64 * nw * 8, np.uint64)
fn(h, buf.ctypes.data_as(ctypes.c_void_p), buf.size)
st = buf.reshape(64, nw, 8).astype(np.int64)
G = pipe.solver.pcg_form()[1]
st = st[:, :G]
names = ["gather m", "spmv", "poll (from start)", "barrier1 (from start)", "recur+M^-1+publish (from b1)",
         "barrier2", "partials published (from b2)"]
valid = (st[1:, :, 0] > 0)
print(f"workgroups {G}, iterations with stamps {int(valid.any(axis=1).sum())}")
def stat(x, label):
    x = x[valid]
    print(f"  {label:32s} median {np.median(x):7.0f}  p10 {np.percentile(x, 10):7.0f}  p90 {np.percentile(x, 90):7.0f}")
s = st[1:]
stat(s[:, :, 1] - s[:, :, 0], "gather m")
stat(s[:, :, 2] - s[:, :, 1], "spmv")
stat(s[:, :, 3] - s[:, :, 0], "poll done (from start)")
stat(s[:, :, 4] - s[:, :, 0], "barrier1 (from start)")
stat(s[:, :, 5] - s[:, :, 4], "recur+M^-1+publish (from b1)")
stat(s[:, :, 6] - s[:, :, 5], "barrier2")
stat(s[:, :, 7] - s[:, :, 6], "partials published (from b2)")
it_len = np.diff(st[:, :, 0], axis=0)[1:]
print(f"  iteration (start to start)       median {np.median(it_len[it_len > 0]):7.0f} cycles")
