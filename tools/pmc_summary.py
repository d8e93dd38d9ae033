"""Per-launch HBM traffic of the roofline kernels from the rocprofv3 PMC CSVs written by
tools/pmc_traffic.sh -> JSON (bench.py reads it into roofline.traffic).

Correction (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE reports half the bytes of
16-B/lane coalesced reads, so traffic = 2 x FETCH_SIZE + WRITE_SIZE (both reported in KB).

  python tools/pmc_summary.py gpurun_out profiles/r05_pmc_traffic.json

The workload the counters were collected on is taken from the bench line the profiled run printed
(gpurun_out/pmc_FETCH_SIZE.log); bench.py uses `traffic` only when that workload equals its own.
"""
import collections
import csv
import json
import os
import sys

import numpy as np

KERNELS = {"k_pcg_iter": ("ofx::k_pcg_iter<true, false",), "k_as_apply": ("ofx::k_as_apply<true",),
           "k_as_iter": ("ofx::k_as_iter<false",), "k_as_w0": ("ofx::k_as_w0<true",),
           "k_as_proj2": ("ofx::k_as_proj2<",), "k_pcg_proj": ("ofx::k_pcg_proj<",),
           "k_as_invert": ("ofx::k_as_invert(",),
           "k_integrate_warp": ("ofx::k_integrate_pal4<true>", "ofx::k_integrate<true, true"),
           "k_assemble": ("ofx::k_assemble(",), "k_terms": ("ofx::k_terms(",),
           "k_brick_cull": ("ofx::k_brick_cull(ofx::BrickGeom, ofx::BrickDiv",), "k_tile_max": ("ofx::k_tile_max(",)}


def workload(d):
    try:
        for line in open(os.path.join(d, "pmc_FETCH_SIZE.log")):
            if line.startswith("{"):
                return json.loads(line)["config"]["workload"]
    except (OSError, ValueError, KeyError):
        pass
    return None


def main(d, out):
    res = {"method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), median over dispatches; "
                     "bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE half-count correction)",
           "workload": workload(d), "kernels": {}}
    vals = collections.defaultdict(dict)
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        rows = list(csv.DictReader(open(os.path.join(d, f"pmc_{c}", "run_counter_collection.csv"))))
        for key, pats in KERNELS.items():
            v = [float(r["Counter_Value"]) for r in rows if any(p in r["Kernel_Name"] for p in pats)]
            if v:
                vals[key][c] = (float(np.median(v)), len(v))
    for key, v in vals.items():
        if "FETCH_SIZE" in v and "WRITE_SIZE" in v:
            fb, wb = v["FETCH_SIZE"][0] * 1024, v["WRITE_SIZE"][0] * 1024
            res["kernels"][key] = {"fetch_size_bytes_raw": fb, "write_size_bytes": wb, "traffic_bytes": 2 * fb + wb,
                                   "dispatches": v["FETCH_SIZE"][1]}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
