set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread \
  "tests/test_gpu_schwarz.py::test_one_launch_iteration_is_bitwise_the_two_launch_form" > gpurun_out/r06c8_one.log 2>&1
rc=$?; grep -E "bit for bit|passed|failed|Error|assert" gpurun_out/r06c8_one.log | tail -6; [ $rc -eq 0 ] || exit $rc
OFX_LIB=tools/stampslib/libofx_stamps.so timeout -k 10 180 python tools/as_iter_stamps.py > gpurun_out/r06c8_stamps.log 2>&1; rc=$?; head -10 gpurun_out/r06c8_stamps.log | tail -9; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1 0; do
  OFX_AS_ONE=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06c8_bench_$v.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/r06c8_bench_$v.log').read().strip().splitlines()[-1]); r=d['roofline']; print('one=$v', round(d['value'],1), round(d['breakdown_ms']['solve'],3), r['iterations_per_frame'], r['launches_per_frame'], round(r['avg_launch_us'],3), round(r['frac'],3))"
done
