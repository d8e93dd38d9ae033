set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_schwarz.py tests/test_gpu_stoprule.py tests/test_gpu_moose.py -rA > gpurun_out/r06c17_tests.log 2>&1 || { tail -40 gpurun_out/r06c17_tests.log; exit 1; }
tail -1 gpurun_out/r06c17_tests.log
OFX_LIB=tools/stampslib/libofx_stamps.so timeout -k 10 180 python tools/as_iter_stamps.py > gpurun_out/r06c17_stamps.log 2>&1 || exit $?
tail -5 gpurun_out/r06c17_stamps.log
ROUNDS=3 bash tools/ab_libs.sh p2 cur
VAR=OFX_PCG_RATIO ROUNDS=2 bash tools/ab_env.sh 2 1 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof17 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 10 > $R/gpurun_out/r06c17_rocprof.log 2>&1
cd $R
python tools/kstats.py gpurun_out/prof17/run_results.db > gpurun_out/r06c17_kstats.txt
rm -rf gpurun_out/prof17
grep -i "invert\|k_as_w0\|proj2" gpurun_out/r06c17_kstats.txt
