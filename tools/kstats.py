"""Per-kernel stats (calls, total/avg/min/max ns) from a rocprofv3 rocpd SQLite database.

  python tools/kstats.py gpurun_out/prof/run_results.db [--csv out.csv]
"""
import sqlite3
import sys


def stats(db):
    c = sqlite3.connect(db)
    q = """select s.kernel_name, count(*), sum(d.end-d.start), avg(d.end-d.start), min(d.end-d.start), max(d.end-d.start)
           from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
           group by s.kernel_name order by sum(d.end-d.start) desc"""
    return list(c.execute(q))


if __name__ == "__main__":
    rows = stats(sys.argv[1])
    tot = sum(r[2] for r in rows)
    lines = ["Name,Calls,TotalDurationNs,AverageNs,MinNs,MaxNs,Percentage"]
    for n, k, s, a, mn, mx in rows:
        lines.append(f'"{n}",{k},{s},{a:.1f},{mn},{mx},{100 * s / tot:.3f}')
    out = "\n".join(lines)
    if "--csv" in sys.argv:
        open(sys.argv[sys.argv.index("--csv") + 1], "w").write(out + "\n")
    for n, k, s, a, mn, mx in rows[:40]:
        print(f"{n[:70]:70s} {k:7d} {s / 1e6:9.3f} ms {a / 1e3:9.2f} us")
