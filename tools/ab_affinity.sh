#!/bin/bash
# A/B of the host process's CPU placement on the launch-bound PCG loop (interleaved runs on one box):
# pinned to the CPUs of the GPU's NUMA node (rocm-smi topology) vs pinned to the other node.
# Writes gpurun_out/ab_aff/*.
set -e
out=gpurun_out/ab_aff; rm -rf $out; mkdir -p $out
node=$(rocm-smi --showtoponuma 2>/dev/null | sed -n 's/.*(Topology) Numa Node: *\([0-9]*\).*/\1/p' | head -1)
loc=$(python -c "
import glob,os
n=int('$node'); a=sorted(os.sched_getaffinity(0))
on=lambda c: os.path.exists(f'/sys/devices/system/cpu/cpu{c}/node{n}')
print(','.join(str(c) for c in a if on(c)), ','.join(str(c) for c in a if not on(c)))")
set -- $loc
echo "gpu numa node $node; local $1; remote $2" > $out/probe.txt
for r in 1 2 3; do
  timeout -k 10 150 taskset -c $1 python bench.py --no-cpu-baseline --json-out $out/loc_$r.json > $out/loc_$r.txt 2>&1
  timeout -k 10 150 taskset -c $2 python bench.py --no-cpu-baseline --json-out $out/rem_$r.json > $out/rem_$r.txt 2>&1
done
cat $out/probe.txt
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/ab_aff/*.json")):
    d = json.load(open(f)); print(f, round(d["value"], 1), round(d["roofline"]["avg_launch_us"], 3))
PY
