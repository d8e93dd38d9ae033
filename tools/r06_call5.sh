# one-launch iteration: bitwise check, A/B bench (one / two launches), kernel trace of the one-launch bench
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread \
  "tests/test_gpu_schwarz.py::test_one_launch_iteration_is_bitwise_the_two_launch_form" > gpurun_out/r06c5_one.log 2>&1
rc=$?; grep -E "bit for bit|passed|failed|Error|assert" gpurun_out/r06c5_one.log | tail -6; [ $rc -eq 0 ] || exit $rc
for v in "1 1" "1 0" "0 1" "1 1" "1 0" "0 1"; do
  set -- $v
  OFX_AS_ONE=$1 OFX_AS_ROWSPLIT=$2 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06c5_bench_$1$2.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/r06c5_bench_$1$2.log').read().strip().splitlines()[-1]); r=d['roofline']; print('one=$1 rowsplit=$2', round(d['value'],1), round(d['breakdown_ms']['solve'],3), r['iterations_per_frame'], r['launches_per_frame'], round(r['avg_launch_us'],3), round(r['frac'],3))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r06c5_prof -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/r06c5_rocprof.log 2>&1 || exit $?
cd $R
python tools/kstats.py gpurun_out/r06c5_prof/run_results.db > gpurun_out/r06c5_kstats.txt 2>&1 || true
head -24 gpurun_out/r06c5_kstats.txt
rm -rf gpurun_out/r06c5_prof
