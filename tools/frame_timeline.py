"""One frame's GPU timeline from a rocprofv3 rocpd database (tuning tool): every dispatch between two
consecutive warped-integrate launches with its start offset, duration and the idle gap before it, plus
per-kernel totals and the frame's busy / idle split.

  python tools/frame_timeline.py gpurun_out/prof/run_results.db [frame_index]
"""
import sqlite3
import sys
from collections import defaultdict


def dispatches(db):
    c = sqlite3.connect(db)
    q = """select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d
           join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start"""
    return list(c.execute(q))


def short(n):
    n = n.replace(".kd", "")
    for key in ("k_pcg_iter", "k_integrate_pal4", "k_integrate", "k_assemble", "k_terms", "k_pcg_proj2", "k_pcg_proj",
                "k_pcg_w0", "k_pcg_prep", "k_step", "copyBuffer", "fillBuffer"):
        if key in n:
            return key
    return n[:40]


def main():
    rows = dispatches(sys.argv[1])
    which = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    marks = [i for i, r in enumerate(rows) if "k_integrate" in r[0] and ("ILb1E" in r[0] or "pal4" in r[0])]
    a, b = marks[which], marks[which + 1]
    frame = rows[a + 1:b + 1]
    t0 = rows[a][2]
    busy = sum(e - s for _, s, e in frame)
    span = frame[-1][2] - t0
    tot = defaultdict(lambda: [0, 0, 0])
    prev = t0
    out = []
    for n, s, e in frame:
        k = short(n)
        tot[k][0] += 1
        tot[k][1] += e - s
        tot[k][2] += max(0, s - prev)
        out.append(f"{(s - t0) / 1e3:9.2f} us  {(e - s) / 1e3:8.2f} us  gap {(s - prev) / 1e3:7.2f}  {k}")
        prev = e
    print(f"frame span {span / 1e3:.1f} us, busy {busy / 1e3:.1f} us, idle {(span - busy) / 1e3:.1f} us, "
          f"{len(frame)} dispatches")
    for k, (n, d, g) in sorted(tot.items(), key=lambda x: -x[1][1] - x[1][2]):
        print(f"  {k:24s} n={n:5d} busy {d / 1e3:9.1f} us  gaps-before {g / 1e3:8.1f} us")
    if "-v" in sys.argv:
        print("\n".join(out))


if __name__ == "__main__":
    main()
