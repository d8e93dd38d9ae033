# Round measurement on the GPU box: PMC traffic (separate counter passes) -> kernel-trace stats -> full bench
# line with the CPU baseline. Everything lands in gpurun_out/ (copied into profiles/ afterwards).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/pmc_traffic.sh
python tools/pmc_summary.py gpurun_out gpurun_out/r01_pmc_traffic.json
cp gpurun_out/r01_pmc_traffic.json profiles/r01_pmc_traffic.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_final -o run -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/bench_rocprof.log 2>&1
cd $R
grep '"metric"' gpurun_out/bench_rocprof.log | tail -1 > gpurun_out/r01_bench_under_rocprof.json
python tools/kstats.py gpurun_out/prof_final/run_results.db --csv gpurun_out/r01_bench_kernel_stats.csv > gpurun_out/kstats.txt; head -12 gpurun_out/kstats.txt
timeout -k 10 600 python bench.py > gpurun_out/bench_full.log 2>&1
tail -1 gpurun_out/bench_full.log > gpurun_out/r01_bench.json
cat gpurun_out/r01_bench.json
