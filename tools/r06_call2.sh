# Round-6 GPU call: the one-launch Schwarz iteration (k_as_iter) against the two-launch form, bit for bit; the stop-rule
# matrix; then an A/B bench (one-launch default vs OFX_AS_ONE=0) in the driver's form.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest -x -v -s --timeout 200 --timeout-method thread \
  "tests/test_gpu_schwarz.py::test_one_launch_iteration_is_bitwise_the_two_launch_form" > gpurun_out/r06c2_one.log 2>&1
rc=$?; grep -E "bit for bit|passed|failed|Error|assert" gpurun_out/r06c2_one.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread tests/test_gpu_schwarz.py \
  tests/test_gpu_stoprule.py > gpurun_out/r06c2_tests.log 2>&1
rc=$?; grep -E "inside|passed|failed|Error" gpurun_out/r06c2_tests.log | tail -30; [ $rc -eq 0 ] || exit $rc
for m in 1 0 1 0; do
  OFX_AS_ONE=$m timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06c2_bench_one$m.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/r06c2_bench_one$m.log').read().strip().splitlines()[-1]); r=d['roofline']; print('one=$m', round(d['value'],1), round(d['breakdown_ms']['solve'],3), r['iterations_per_frame'], r['launches_per_frame'], round(r['avg_launch_us'],3), round(r['frac'],3))"
done
