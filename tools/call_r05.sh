set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_moose.py tests/test_gpu_golden_gn.py tests/test_gpu_ops.py tests/test_gpu_api.py tests/test_gpu_prefetch.py -x -v --timeout 200 --timeout-method thread > gpurun_out/c1_tests.log 2>&1; rc=$?; tail -5 gpurun_out/c1_tests.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --moose --steps 10 --warmup 2 > gpurun_out/c1_moose.log 2>&1 || exit $?
tail -1 gpurun_out/c1_moose.log | cut -c1-1500
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/c1_bench.log 2>&1 || exit $?
tail -1 gpurun_out/c1_bench.log | cut -c1-900
