"""Runtime-glue dispatches inside bench.py's timed frames, from a rocprofv3 --kernel-trace database.

  python tools/rocclr_in_loop.py gpurun_out/prof/run_results.db --warmup 3 --steps 10

The timed frames are the ones whose warped integrate (k_integrate_pal4, one per frame) is the (warmup+1)-th .. (warmup+
steps)-th: every dispatch that starts after the warmup's last integrate ends and before the last timed integrate ends
is counted per kernel name; rocclr fill / copy blits and torch / rocprim kernels are listed per frame.
"""
import argparse
import collections
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--warmup", type=int, default=3)
ap.add_argument("--steps", type=int, default=10)
a = ap.parse_args()
c = sqlite3.connect(a.db)
rows = list(c.execute("""select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d
                         join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start"""))
pal = [r for r in rows if "k_integrate_pal4" in r[0]]
t0, t1 = pal[a.warmup - 1][2], pal[a.warmup + a.steps - 1][2]
cnt = collections.Counter(r[0] for r in rows if t0 < r[1] <= t1)
glue = {k: v for k, v in cnt.items() if "rocclr" in k or "at::" in k or "at6native" in k or "rocprim" in k}
print(f"timed frames {a.steps}: {sum(cnt.values())} dispatches, {sum(cnt.values()) / a.steps:.1f} per frame")
for k, v in sorted(glue.items(), key=lambda x: -x[1]):
    print(f"  {v / a.steps:6.2f} per frame  {k[:100]}")
print(f"  glue total {sum(glue.values()) / a.steps:.2f} per frame")
