# GPU check of the overlapping Schwarz preconditioner (OFX_PRECOND=as): its parity tests, the whole GPU suite with it
# forced, then a bench A/B against the cluster block Jacobi (100 frames, alternating, one box).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_schwarz.py \
  > gpurun_out/as_tests.log 2>&1; rc=$?
grep -h "Schwarz:\|Schwarz \|passed\|failed\|Max relative" gpurun_out/as_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
OFX_PRECOND=as timeout -k 10 600 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/ \
  > gpurun_out/as_suite.log 2>&1; rc=$?
tail -15 gpurun_out/as_suite.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for i in 1 2; do
  for v in bj as; do
    OFX_PRECOND=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 --warmup 5 > gpurun_out/as_$v$i.json 2> gpurun_out/as_$v$i.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/as_$v$i.json').read().strip().splitlines()[-1]); b=d['breakdown_ms']; r=d['roofline']; print('$v', round(d['value'],1), b.get('pcg_iters_per_frame'), r.get('launches_per_frame'), r.get('avg_launch_us'))"
  done
done
