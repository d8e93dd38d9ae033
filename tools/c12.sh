# Round check after the auto preconditioner: whole GPU suite + smoke, config 2 / 3 lines
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/ > gpurun_out/c12_suite.log 2>&1; rc=$?
tail -4 gpurun_out/c12_suite.log
if [ $rc -ne 0 ]; then grep -h "FAILED\|Error" gpurun_out/c12_suite.log | head -20; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/c12_smoke.log 2>&1 || { tail -20 gpurun_out/c12_smoke.log; exit 1; }
tail -1 gpurun_out/c12_smoke.log
for c in 2 3; do
  timeout -k 10 400 python bench.py --config $c --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/c12_config$c.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/c12_config$c.log').read().strip().splitlines()[-1]); r=d['roofline']; print($c, round(d['value'],1), r['iterations_per_frame'], r['launches_per_frame'], r['preconditioner']['schwarz'])"
done
