"""Summary of tools/pmc_valu.sh: per kernel the mean per dispatch of each SQ counter, and the derived shares
(VALU-busy = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES, parked = SQ_WAIT_ANY / SQ_WAVE_CYCLES; both in quad-cycles,
per wave summed over the chip).

  python tools/pmc_valu_summary.py gpurun_out/pmc_valu/run_counter_collection.csv [out.json]
"""
import collections
import csv
import json
import re
import sys


def main(path, out=None):
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows:
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, d in agg.items():
        m = {c: sum(v) / len(v) for c, v in d.items()}
        m["dispatches"] = max(len(v) for v in d.values())
        wc = m.get("SQ_WAVE_CYCLES", 0.0)
        if wc:
            m["valu_busy_share"] = m.get("SQ_ACTIVE_INST_VALU", 0.0) / wc
            m["parked_share"] = m.get("SQ_WAIT_ANY", 0.0) / wc
        if m.get("SQ_WAVES"):
            m["valu_insts_per_wave"] = m.get("SQ_INSTS_VALU", 0.0) / m["SQ_WAVES"]
        res[k] = m
    txt = json.dumps(res, indent=1)
    if out:
        open(out, "w").write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main(*sys.argv[1:])
