# In-box A/B of the preconditioner refresh threshold on the default bench (100 frames each, alternating, two rounds)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
for i in 1 2; do
  for v in 0.1 0.2 0.4 0; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 --warmup 5 --gn precond_rot_tol=$v > gpurun_out/rt_$v$i.json 2> gpurun_out/rt_$v$i.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/rt_$v$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', round(d['value'],1), round(d['ms_per_step'],4), r.get('iterations_per_frame'), r.get('launches_per_frame'), round(r.get('avg_launch_us'),3))"
  done
done
