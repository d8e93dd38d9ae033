"""Tuning study (not product): per-phase clock stamps of the PCG iteration kernel on the bench workload.

Needs the stamps build: python -c "from occlusionfusion_amd import build; build.build(out='tools/bin/libofx_stamps.so',
defines=['OFX_STAMPS'])", then OFX_LIB=tools/bin/libofx_stamps.so python tools/pcg_stamps.py
Phases per wave (s_memtime cycles): 1 trip 1 | 2 scalars | 3 trip 2 + products | 4 barrier + row sums |
5 recurrences + stores | 6 barrier + M⁻¹ apply + m store | 7 wave sums + partial stores.
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

assert "stamps" in _lib.LIB_PATH, "run with OFX_LIB=tools/bin/libofx_stamps.so"
fn = _lib.lib.ofx_gn_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
fn.restype = ctypes.c_int32
dev = torch.device("cuda", 0)
seq = S.SyntheticSequence.build(2000, seed=3)
D = int(os.environ.get("DIMS", "128"))
pipe = FusionPipeline(seq, (-D * 0.002, -D * 0.002, 0.5), 0.004, (D, D, D), device=dev)
frames = [pipe.prepare(t) for t in range(8)]
pipe.integrate_source(frames[0])
for t in range(1, 6):
    pipe.step(frames[t], t)
torch.cuda.synchronize()
h = pipe.solver._h
fn(h, None, 0)                      # allocate + clear
he = _lib.lib.ofx_gn_host_enqueue
he.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
us, ne = ctypes.c_double(), ctypes.c_int64()
he(h, ctypes.byref(us), ctypes.byref(ne))
import time
t0 = time.perf_counter()
pipe.step(frames[6], 6)
torch.cuda.synchronize()
t1 = time.perf_counter()
he(h, ctypes.byref(us), ctypes.byref(ne))
print(f"frame wall {1e3 * (t1 - t0):.2f} ms; host enqueue of {ne.value} PCG launches {us.value / 1e3:.2f} ms "
      f"({us.value / max(1, ne.value):.2f} us each)")
nw = pipe.solver.info()[4] // 8
buf = np.zeros(64 * nw * 8, np.uint64)
fn(h, buf.ctypes.data_as(ctypes.c_void_p), buf.size)
st = buf.reshape(64, nw, 8).astype(np.int64)
ok = (st > 0).all(axis=2)
d = np.diff(st, axis=2)[ok]          # (samples, 7) cycles per phase
print(f"waves {nw}, sampled (iteration, wave) pairs {d.shape[0]}")
names = ["trip1", "scalars", "trip2+prod", "bar+rowsum", "recur+store", "bar+apply", "sums+part"]
for k, nme in enumerate(names):
    x = d[:, k]
    print(f"  {nme:12s} median {np.median(x):7.0f} cyc  p10 {np.percentile(x, 10):7.0f}  p90 {np.percentile(x, 90):7.0f}")
tot = st[:, :, 7] - st[:, :, 0]
print(f"  total        median {np.median(tot[ok]):7.0f} cyc  p90 {np.percentile(tot[ok], 90):7.0f}")
# cross-wave spread of entry/exit within an iteration (if the counters agree across CUs)
for it in (5, 20, 40):
    if ok[it].all():
        e0, e7 = st[it, :, 0], st[it, :, 7]
        print(f"  iter {it}: entry spread {e0.max() - e0.min()} cyc, exit spread {e7.max() - e7.min()} cyc, "
              f"first entry -> last exit {e7.max() - e0.min()} cyc")
