set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r02_gputest4.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r02_gputest4.log
[ $rc -le 1 ] || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ab7 -o run -- python3 $R/tools/int_ab.py 3 > $R/gpurun_out/ab7.log 2>&1; echo "ab rc=$?"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_bench7 -o run -- python3 $R/bench.py --steps 30 --no-cpu-baseline > $R/gpurun_out/bench7_prof.log 2>&1; echo "benchprof rc=$?"
cd $R
python tools/kstats.py gpurun_out/prof_ab7/run_results.db | grep -i integrate
python tools/frame_timeline.py gpurun_out/prof_bench7/run_results.db 10 > gpurun_out/timeline7.txt; head -30 gpurun_out/timeline7.txt
