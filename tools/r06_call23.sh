set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_schwarz.py tests/test_gpu_configs.py > gpurun_out/r06c23_tests.log 2>&1 || { tail -30 gpurun_out/r06c23_tests.log; exit 1; }
tail -1 gpurun_out/r06c23_tests.log
timeout -k 10 400 python bench.py --config 4 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r06c23_config4.log 2>&1 || exit $?
tail -1 gpurun_out/r06c23_config4.log > gpurun_out/r06_bench_config4.json
python -c "import json; d=json.loads(open('gpurun_out/r06_bench_config4.json').read()); r=d['roofline']; print('config4', round(d['value'],1), r['iterations_per_frame'], r['launches_per_frame'], round(r['avg_launch_us'],3), r['preconditioner'])"
