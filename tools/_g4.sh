set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r02_gputest3.log 2>&1; rc=$?; echo "tests rc=$rc"
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 300 python tools/int_ab.py 3 > gpurun_out/r02_int_ab.log 2>&1; echo "ab rc=$?"
  timeout -k 10 300 python bench.py --steps 100 --no-cpu-baseline > gpurun_out/r02_bench_pal4.log 2>&1; echo "bench rc=$?"
fi
