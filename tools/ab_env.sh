#!/bin/bash
# A/B of one environment variable's values on bench.py (current libofx.so), alternating, ROUNDS rounds:
#   VAR=OFX_PCG_RATIO ROUNDS=3 bash tools/ab_env.sh 2 1 0
set -e
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in "$@"; do
    env $VAR=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-40} > gpurun_out/abe.json 2>/dev/null
    python -c "import json; d=json.loads(open('gpurun_out/abe.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$VAR=$v', round(d['value'],1), round(r['iterations_per_frame'],1), round(r['launches_per_frame'],1), round(r['avg_launch_us'],3), round(d['breakdown_ms']['solve'],3))"
  done
done
