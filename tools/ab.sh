# A/B of the working tree's libofx.so against tools/bin/libofx_base.so on one box (bench.py, 100 frames,
# alternating): prints value / pcg iterations per run.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for i in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export OFX_LIB=$R/tools/bin/libofx_base.so; else unset OFX_LIB; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/ab_$v$i.json 2> gpurun_out/ab_$v$i.err
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$v$i.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['breakdown_ms']['pcg_iters_per_frame'], d['roofline']['avg_launch_us'])"
  done
done
