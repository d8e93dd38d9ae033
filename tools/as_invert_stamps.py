"""Tuning study (not product): phase clock stamps of the Schwarz subdomain inversion (k_as_invert) on the bench workload.

Needs the stamps build: python -c "from occlusionfusion_amd import build; build.build(out='tools/stampslib/libofx_stamps.so',
defines=['OFX_STAMPS'])", then OFX_LIB=tools/stampslib/libofx_stamps.so python tools/as_invert_stamps.py
Phases (thread 0 of each subdomain's workgroup, s_memtime cycles): 1 tables + A gather | 2 block Gauss-Jordan |
3 scales + fp16 margin | 4 LDS image | 5 slab rows.
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

assert "stamps" in _lib.LIB_PATH, "run with OFX_LIB=tools/stampslib/libofx_stamps.so"
fn = _lib.lib.ofx_gn_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64]
fn.restype = ctypes.c_int32
dev = torch.device("cuda", 0)
c = S.BASELINE_CONFIGS[3]
seq = S.config_sequence(3, None, rank=0, device=dev)
D = c["dims"]
pipe = FusionPipeline(seq, c["origin"], c["voxel"], (D, D, D), device=dev)
frames = [pipe.prepare(t) for t in range(6)]
pipe.integrate_source(frames[0])
for t in range(1, 4):
    pipe.step(frames[t], t)
torch.cuda.synchronize()
h = pipe.solver._h
fn(h, None, 0)                      # allocate + clear
pipe.step(frames[4], 4)
torch.cuda.synchronize()
nw = pipe.solver.info()[4] // 8
buf = np.zeros(64 * nw * 8, np.uint64)
fn(h, buf.ctypes.data_as(ctypes.c_void_p), buf.size)
st = buf.reshape(64, nw, 8)[63, :, :6].astype(np.int64)
ok = (st > 0).all(axis=1)
d = np.diff(st[ok], axis=1)
print(f"subdomains {nw}, stamped {int(ok.sum())}")
for k, nme in enumerate(["tables+A", "gauss-jordan", "scale+margin", "lds image", "slab rows"]):
    x = d[:, k]
    print(f"  {nme:14s} median {np.median(x):8.0f} cyc  p90 {np.percentile(x, 90):8.0f}")
ex = buf.reshape(64, nw, 8)[63, :, 6:].astype(np.int64)[ok]
if (ex > 0).any():   # the MFMA form: cycles spent in the pivot-block inversions / the tile updates, summed over panels
    print(f"  (MFMA form) pivot blocks {np.median(ex[:, 0]):8.0f} cyc, V + update {np.median(ex[:, 1]):8.0f} cyc")
tot = st[ok, 5] - st[ok, 0]
print(f"  total          median {np.median(tot):8.0f} cyc  p90 {np.percentile(tot, 90):8.0f}; "
      f"first entry -> last exit {st[ok, 5].max() - st[ok, 0].min()} cyc")
