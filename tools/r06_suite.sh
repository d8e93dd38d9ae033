# the whole GPU suite + smoke on the current tree, then the bench in the driver's form
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/ > gpurun_out/r06_suite.log 2>&1; rc=$?
tail -3 gpurun_out/r06_suite.log
if [ $rc -ne 0 ]; then grep -h "FAILED\|Error" gpurun_out/r06_suite.log | head -20; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06_smoke.log 2>&1 || { tail -20 gpurun_out/r06_smoke.log; exit 1; }
tail -1 gpurun_out/r06_smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r06_bench_driver.log 2>&1 || exit $?
tail -1 gpurun_out/r06_bench_driver.log | cut -c1-600
