# A/B on one box of the working tree's libofx.so with an environment switch: base = "$AB_ENV" set (e.g.
# AB_ENV=OFX_PCG_W1=1), new = unset; bench.py, 100 frames, alternating, two rounds
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for i in 1 2; do
  for v in base new; do
    if [ $v = base ]; then E="env $AB_ENV"; else E=""; fi
    timeout -k 10 300 $E python bench.py --no-cpu-baseline > gpurun_out/ab_$v$i.json 2> gpurun_out/ab_$v$i.err
    python -c "import json; d=json.loads(open('gpurun_out/ab_$v$i.json').read().strip().splitlines()[-1]); print('$v', round(d['value'],2), d['breakdown_ms']['pcg_iters_per_frame'], round(d['roofline']['avg_launch_us'],3))"
  done
done
