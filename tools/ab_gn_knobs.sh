# In-box A/B of PCG chunk knobs on the default bench (100 frames each, alternating, two rounds)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
for i in 1 2; do
  for v in base t4 t4r1 t2r1; do
    E="OFX_NONE=1"
    case $v in t4) E="OFX_PCG_TOPUP=4";; t4r1) E="OFX_PCG_TOPUP=4 OFX_PCG_RATIO=1";; t2r1) E="OFX_PCG_TOPUP=2 OFX_PCG_RATIO=1";; esac
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 --warmup 5 > gpurun_out/kn_$v$i.json 2> gpurun_out/kn_$v$i.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/kn_$v$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', round(d['value'],1), round(d['ms_per_step'],4), r.get('iterations_per_frame'), r.get('launches_per_frame'), round(r.get('avg_launch_us'),3))"
  done
done
