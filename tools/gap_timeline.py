"""Tuning (not product): GPU idle gaps of a bench run from a rocprofv3 --kernel-trace CSV — the sum of the gaps
between consecutive dispatches on the device, classified by the (previous, next) kernel pair, over the timed frames
(the last `frames` integrate launches delimit them). Under the tracer every dispatch gets its own overhead, so the
absolute numbers are inflated; the split between classes is what this is for.

  python tools/gap_timeline.py run_kernel_trace.csv [frames=20]
"""
import collections
import csv
import re
import sys


def short(n):
    m = re.search(r"(k_\w+)", n)
    return m.group(1) if m else n.split("(")[0][-30:]


def main(path, frames=20):
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in csv.DictReader(open(path))]
    rows.sort()
    ints = [i for i, r in enumerate(rows) if r[2] == "k_integrate_pal4"]
    # timed region: from after the integrate that precedes the timed frames to the last frame's integrate; the bench's
    # isolated integrate launches (20 after the loop) are excluded by taking the frames' integrates before them
    loop_ints = [i for i in ints if any(r[2] == "k_pcg_iter" for r in rows[max(0, i - 40):i])]   # after a solve
    sel = loop_ints[-frames - 1:]
    a, b = sel[0], sel[-1]
    busy = collections.Counter()
    gaps = collections.Counter()
    cnt = collections.Counter()
    for i in range(a + 1, b + 1):
        s, e, n = rows[i]
        busy[n] += e - s
        g = s - rows[i - 1][1]
        if g > 0:
            key = (rows[i - 1][2], n)
            gaps[key] += g
            cnt[key] += 1
    span = rows[b][1] - rows[a][1]
    tb, tg = sum(busy.values()), sum(gaps.values())
    print(f"frames {len(sel) - 1}: span {span / 1e3 / (len(sel) - 1):.1f} us/frame, busy {tb / 1e3 / (len(sel) - 1):.1f}, "
          f"gaps {tg / 1e3 / (len(sel) - 1):.1f} us/frame")
    print("busy per frame (us):")
    for n, v in busy.most_common(12):
        print(f"  {n:28s} {v / 1e3 / (len(sel) - 1):8.1f}")
    print("gaps per frame (us) by (previous -> next):")
    for k, v in gaps.most_common(16):
        print(f"  {k[0]:22s} -> {k[1]:22s} {v / 1e3 / (len(sel) - 1):8.1f}  ({cnt[k] / (len(sel) - 1):.1f} per frame)")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20)
