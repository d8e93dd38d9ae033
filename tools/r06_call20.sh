set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -s -m gpu --timeout 200 --timeout-method thread tests/test_gpu_schwarz.py -k "mfma or gn_2k_chain or moose" > gpurun_out/r06c20_tests.log 2>&1; rc=$?
grep -h "PCG\|passed\|failed\|Error\|error" gpurun_out/r06c20_tests.log | head -20
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof20 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 10 > $R/gpurun_out/r06c20_rocprof.log 2>&1
cd $R
python tools/kstats.py gpurun_out/prof20/run_results.db > gpurun_out/r06c20_kstats.txt
rm -rf gpurun_out/prof20
grep -i "invert" gpurun_out/r06c20_kstats.txt
