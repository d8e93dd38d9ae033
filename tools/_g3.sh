set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r02_gputest2.log 2>&1; rc=$?; echo "tests rc=$rc"
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python bench.py --steps 100 --no-cpu-baseline > gpurun_out/r02_bench_ops.log 2>&1; echo "bench rc=$?"
fi
