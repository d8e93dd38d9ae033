#!/bin/bash
# A/B of several libofx builds (tools/ablib/libofx_<tag>.so and the current one) on bench.py, alternating, two rounds
set -e
for r in $(seq 1 ${ROUNDS:-2}); do
  for L in "$@"; do
    P=tools/ablib/libofx_$L.so; [ "$L" = cur ] && P=occlusionfusion_amd/libofx.so
    OFX_LIB=$P timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 > gpurun_out/abl.json 2>/dev/null
    python -c "import json; d=json.loads(open('gpurun_out/abl.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$L', round(d['value'],1), round(r['iterations_per_frame'],1), round(r['launches_per_frame'],1), round(r['avg_launch_us'],3), round(d['breakdown_ms']['solve'],3))"
  done
done
