# In-box A/B of GN knobs on the default bench (100 frames each, alternating, two rounds): chunk margin, warm start
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
for i in 1 2; do
  for v in base r0 r1 nowarm; do
    E=""; G=""
    case $v in r0) E="OFX_PCG_RATIO=0";; r1) E="OFX_PCG_RATIO=1";; nowarm) G="--gn pcg_warm=0";; esac
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 --warmup 5 $G > gpurun_out/kn_$v$i.json 2> gpurun_out/kn_$v$i.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/kn_$v$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', round(d['value'],1), round(d['ms_per_step'],4), r.get('iterations_per_frame'), r.get('launches_per_frame'), round(r.get('avg_launch_us'),3))"
  done
done
