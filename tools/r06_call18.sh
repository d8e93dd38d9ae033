set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/ > gpurun_out/r06c18_suite.log 2>&1; rc=$?
tail -2 gpurun_out/r06c18_suite.log
if [ $rc -ne 0 ]; then grep -h "FAILED\|Error" gpurun_out/r06c18_suite.log | head -20; exit $rc; fi
ROUNDS=3 bash tools/ab_libs.sh p2 cur
VAR=OFX_PCG_RATIO ROUNDS=2 bash tools/ab_env.sh 2 1 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof18 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 10 > $R/gpurun_out/r06c18_rocprof.log 2>&1
cd $R
python tools/kstats.py gpurun_out/prof18/run_results.db > gpurun_out/r06c18_kstats.txt
rm -rf gpurun_out/prof18
grep -i "invert\|rocclr\|k_as_w0\|proj2" gpurun_out/r06c18_kstats.txt
