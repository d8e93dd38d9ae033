# Round-6 GPU call: the stop-rule matrix and the GN fixture tests, then a driver-form bench line and the moose line.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_stoprule.py \
  tests/test_gpu_golden_gn.py tests/test_gpu_schwarz.py tests/test_gpu_moose.py > gpurun_out/r06c1_tests.log 2>&1
rc=$?; grep -E "inside|passed|failed|Error" gpurun_out/r06c1_tests.log | tail -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06c1_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r06c1_bench.log
timeout -k 10 300 python bench.py --moose --steps 10 --warmup 3 > gpurun_out/r06c1_moose.log 2>&1 || exit $?
tail -1 gpurun_out/r06c1_moose.log
