# GPU check with the Schwarz default: the whole GPU suite + smoke, then a bench A/B against the cluster block Jacobi
# (OFX_PRECOND=bj; 100 frames, alternating, one box) and the driver's 20-frame line.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 600 python -u -m pytest -v -s -m gpu --timeout 300 --timeout-method thread tests/ \
  > gpurun_out/as_suite.log 2>&1; rc=$?
grep -h "Schwarz:\|Schwarz \|passed\|failed\|FAILED" gpurun_out/as_suite.log | tail -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/as_smoke.log 2>&1 || { tail -20 gpurun_out/as_smoke.log; exit 1; }
tail -3 gpurun_out/as_smoke.log
for i in 1 2; do
  for v in bj as; do
    OFX_PRECOND=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 --warmup 5 > gpurun_out/as_$v$i.json 2> gpurun_out/as_$v$i.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/as_$v$i.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; r=d['roofline']; print('$v', round(d['value'],1), b.get('pcg_iters_per_frame'), r.get('launches_per_frame'), r.get('avg_launch_us'), r.get('frac'))"
  done
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/as_driver.json 2> gpurun_out/as_driver.err || exit $?
python -c "import json; d=json.loads(open('gpurun_out/as_driver.json').read().strip().splitlines()[-1]); r=d['roofline']; print('driver', round(d['value'],1), r.get('launches_per_frame'), r.get('iterations_per_frame'), r.get('frac'), d['cpu_baseline']['value'])"
