#!/bin/bash
# tuning sweep: k_pcg_iter waves per workgroup
for w in 1 2 4 1; do
  OFX_PCG_WPB=$w timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/wpb_$w.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/wpb_$w.log').read().strip().splitlines()[-1]);print($w, round(d['value'],2), round(d['roofline']['avg_launch_us'],3))"
done
