#!/bin/bash
# A/B of the untimed warmup length (3 vs 30 frames) on the config-3 bench, interleaved runs on one box.
set -e
out=gpurun_out/ab_warm; rm -rf $out; mkdir -p $out
for r in 1 2 3 4; do
  timeout -k 10 150 python bench.py --no-cpu-baseline --warmup 3 --json-out $out/w3_$r.json > $out/w3_$r.txt 2>&1
  timeout -k 10 150 python bench.py --no-cpu-baseline --warmup 30 --json-out $out/w30_$r.json > $out/w30_$r.txt 2>&1
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/ab_warm/*.json")):
    d = json.load(open(f)); print(f, round(d["value"], 1), round(d["roofline"]["avg_launch_us"], 3),
                                  d["breakdown_ms"]["pcg_iters_per_frame"], d["roofline"]["launches_per_frame"])
PY
