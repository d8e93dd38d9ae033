set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof15 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 30 > $R/gpurun_out/r06c15_rocprof.log 2>&1
cd $R
python tools/kstats.py gpurun_out/prof15/run_results.db --csv gpurun_out/r06c15_kstats.csv > gpurun_out/r06c15_kstats.txt
rm -rf gpurun_out/prof15
head -30 gpurun_out/r06c15_kstats.txt
