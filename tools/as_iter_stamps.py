"""Tuning study (not product): per-phase clock stamps of the one-launch Schwarz iteration (k_as_iter) on a 2k-node frame.

Needs the stamps build: python -c "from occlusionfusion_amd import build; build.build(out='tools/stampslib/libofx_stamps.so',
defines=['OFX_STAMPS'])", then OFX_LIB=tools/stampslib/libofx_stamps.so python tools/as_iter_stamps.py
Stamps of the own-row wave (s_memtime): 0 entry | 1 trip 1 landed | 2 scalars done | 3 barrier 1 (m on S2) |
4 barrier 2 (products) | 5 barrier 3 (recurrences, w image) | 6 end; 7 = the row sums done (after 4).
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
seq = S.SyntheticSequence.build(2000, seed=3)
D = 128
pipe = FusionPipeline(seq, (-D * 0.002, -D * 0.002, 0.5), 0.004, (D, D, D), device=dev)
frames = [pipe.prepare(t) for t in range(8)]
pipe.integrate_source(frames[0])
for t in range(1, 6):
    pipe.step(frames[t], t)
torch.cuda.synchronize()
h = pipe.solver._h
fn(h, None, 0)
pipe.step(frames[6], 6)
torch.cuda.synchronize()
h = pipe.solver._h
nw = pipe.solver.info()[4] // 8
buf = np.zeros(64 * nw * 8, np.uint64)
fn(h, buf.ctypes.data_as(ctypes.c_void_p), buf.size)
st = buf.reshape(64, nw, 8).astype(np.int64)
ok = (st[:, :, :7] > 0).all(axis=2)
print(f"clusters {nw}, sampled (iteration, cluster) pairs {int(ok.sum())}, precond {pipe.solver.precond_info()}")
names = ["trip1", "scalars", "to bar1", "to bar2", "bar3+recur", "tail"]
d = np.diff(st[:, :, :7], axis=2)[ok]
for k, nme in enumerate(names):
    x = d[:, k]
    print(f"  {nme:11s} median {np.median(x):7.0f}  p10 {np.percentile(x, 10):7.0f}  p90 {np.percentile(x, 90):7.0f}")
tot = (st[:, :, 6] - st[:, :, 0])[ok]
print(f"  total       median {np.median(tot):7.0f}  p90 {np.percentile(tot, 90):7.0f}")
s7 = (st[:, :, 7] - st[:, :, 4])[ok & (st[:, :, 7] > 0)]
print(f"  row sums done (from barrier 2): median {np.median(s7):7.0f}")
# spread of entry across clusters in one iteration, and iteration period
for it in (5, 10):
    e = st[it, :, 0][st[it, :, 0] > 0]
    e1 = st[it + 1, :, 0][st[it + 1, :, 0] > 0]
    if e.size and e1.size:
        print(f"  iteration {it}: entry spread {e.max() - e.min()} cycles, next iteration's first entry - this one's "
              f"first {e1.min() - e.min()}, last end {st[it, :, 6].max() - e.min()}")
# per XCD (clusters [x·per, (x+1)·per) run on XCD x: k_as_iter's workgroup mapping): the iteration's span on the XCD's
# clock (s_memtime is per XCD), the latest finisher, and whether the same clusters finish last every iteration
per = (nw + 7) // 8
late = np.zeros(nw)
spans, ent, tot_c = [], [], []
for it in range(1, 60):
    for x in range(8):
        cl = np.arange(x * per, min((x + 1) * per, nw))
        s = st[it, cl]
        good = (s[:, 0] > 0) & (s[:, 6] > 0)
        if good.sum() < len(cl):
            continue
        e0 = s[:, 0].min()
        spans.append(s[:, 6].max() - e0)
        ent.append(np.percentile(s[:, 0] - e0, 90))
        late[cl[np.argmax(s[:, 6])]] += 1
        tot_c.append(s[:, 6] - s[:, 0])
if spans:
    print(f"  per-XCD span (first entry -> last end): median {np.median(spans):.0f}, p90 {np.percentile(spans, 90):.0f};"
          f" entry offsets p90 {np.median(ent):.0f}")
    tc = np.array(tot_c)
    print(f"  per-cluster totals: median {np.median(tc):.0f}, max over the XCD median {np.median(tc.max(axis=1)):.0f}")
    top = np.argsort(-late)[:8]
    print("  clusters most often last on their XCD:", [(int(c), int(late[c])) for c in top])
