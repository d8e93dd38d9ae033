set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread \
  "tests/test_gpu_schwarz.py::test_one_launch_iteration_is_bitwise_the_two_launch_form" > gpurun_out/r06c6_one.log 2>&1
rc=$?; grep -E "bit for bit|passed|failed|Error|assert" gpurun_out/r06c6_one.log | tail -6; [ $rc -eq 0 ] || exit $rc
OFX_LIB=tools/stampslib/libofx_stamps.so timeout -k 10 180 python tools/as_iter_stamps.py > gpurun_out/r06c6_stamps.log 2>&1; rc=$?; tail -14 gpurun_out/r06c6_stamps.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r06c6_prof -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/r06c6_rocprof.log 2>&1 || exit $?
cd $R
python tools/kstats.py gpurun_out/r06c6_prof/run_results.db > gpurun_out/r06c6_kstats.txt 2>&1 || true
head -14 gpurun_out/r06c6_kstats.txt; grep -E "k_as_tab|k_as_members" gpurun_out/r06c6_kstats.txt
rm -rf gpurun_out/r06c6_prof
