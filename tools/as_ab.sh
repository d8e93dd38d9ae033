set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
for i in 1 2; do
  for v in bj as as1; do
    W1=0; P=$v; if [ $v = as1 ]; then W1=1; P=as; fi
    OFX_PCG_W1=$W1 OFX_PRECOND=$P timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 --warmup 5 > gpurun_out/as_$v$i.json 2> gpurun_out/as_$v$i.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/as_$v$i.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; r=d['roofline']; print('$v', round(d['value'],1), b.get('pcg_iters_per_frame'), r.get('launches_per_frame'), r.get('avg_launch_us'))"
  done
done
