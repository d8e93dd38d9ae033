set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_prefetch.py > gpurun_out/r06c26_tests.log 2>&1 || { tail -30 gpurun_out/r06c26_tests.log; exit 1; }
tail -1 gpurun_out/r06c26_tests.log
for r in 1 2 3; do
  for o in "" "--no-overlap"; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --steps 40 $o > gpurun_out/abo.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/abo.json').read().strip().splitlines()[-1]); r=d['roofline']; print('overlap' if '$o'=='' else 'seq', round(d['value'],1), round(d['ms_per_step'],3), round(d['breakdown_ms']['solve'],3), round(d['breakdown_ms']['integrate'],3), round(r['avg_launch_us'],3))"
  done
done
