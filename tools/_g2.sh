set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -x -v --timeout 600 --timeout-method thread > gpurun_out/r02_gputest1.log 2>&1
echo "tests rc=$?"
timeout -k 10 300 python bench.py --config 2 --steps 30 --no-cpu-baseline > gpurun_out/r02_bench_c2.log 2>&1; echo "c2 rc=$?"
timeout -k 10 300 python bench.py --config 1 --steps 30 --no-cpu-baseline > gpurun_out/r02_bench_c1.log 2>&1; echo "c1 rc=$?"
timeout -k 10 400 python bench.py --config 4 --steps 30 --no-cpu-baseline > gpurun_out/r02_bench_c4.log 2>&1; echo "c4 rc=$?"
timeout -k 10 400 python bench.py --gpus 2 --backend gloo --steps 20 --no-cpu-baseline > gpurun_out/r02_bench_rep2.log 2>&1; echo "rep2 rc=$?"
