#!/bin/bash
# A/B of kernel-argument placement on the launch-bound PCG loop (same box, interleaved runs):
# default vs HIP_FORCE_DEV_KERNARG=1 (kernarg segments in device memory). Writes gpurun_out/ab_kernarg/*.json.
set -e
out=gpurun_out/ab_kernarg; mkdir -p $out
for r in 1 2; do
  timeout -k 10 150 python bench.py --no-cpu-baseline --json-out $out/base_$r.json > $out/base_$r.txt 2>&1
  HIP_FORCE_DEV_KERNARG=1 timeout -k 10 150 python bench.py --no-cpu-baseline --json-out $out/dev1_$r.json > $out/dev1_$r.txt 2>&1
  HIP_FORCE_DEV_KERNARG=0 timeout -k 10 150 python bench.py --no-cpu-baseline --json-out $out/dev0_$r.json > $out/dev0_$r.txt 2>&1
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/ab_kernarg/*.json")):
    d = json.load(open(f)); print(f, round(d["value"], 1), round(d["roofline"]["avg_launch_us"], 3))
PY
