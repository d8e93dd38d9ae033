# A/B: prefetch lead 1 / 2 (GN steps of the current solve the next frame's setup overlaps) and the later-step chunk
# margin 1 (OFX_PCG_RATIO=1) against the defaults, bench 100 frames each, alternating, three rounds
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in base lead2 r1; do
    E="OFX_NONE=1"; [ $v = lead2 ] && E="OFX_PREFETCH_LEAD=2"; [ $v = r1 ] && E="OFX_PCG_RATIO=1"
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 --warmup 5 > gpurun_out/pl_$v$i.json 2> gpurun_out/pl_$v$i.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/pl_$v$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', round(d['value'],1), round(d['ms_per_step'],4), r.get('iterations_per_frame'), r.get('launches_per_frame'), round(r.get('avg_launch_us'),3))"
  done
done
