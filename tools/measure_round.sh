# Round measurement on the GPU box: PMC traffic (separate counter passes) -> kernel-trace stats -> full bench
# line with the CPU baseline (reads the PMC summary just written). Everything lands in gpurun_out/ (copied into
# profiles/ afterwards). Every GPU step has its own time limit; the script stops at the first failure.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${TAG:-r05}
cd $R
bash tools/pmc_traffic.sh
python tools/pmc_summary.py gpurun_out gpurun_out/${TAG}_pmc_traffic.json
cp gpurun_out/${TAG}_pmc_traffic.json profiles/${TAG}_pmc_traffic.json
bash tools/pmc_valu.sh
python tools/pmc_valu_summary.py gpurun_out/pmc_valu/run_counter_collection.csv gpurun_out/${TAG}_pmc_valu.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_final -o run -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/bench_rocprof.log 2>&1
cd $R
grep '"metric"' gpurun_out/bench_rocprof.log | tail -1 > gpurun_out/${TAG}_bench_under_rocprof.json
python tools/kstats.py gpurun_out/prof_final/run_results.db --csv gpurun_out/${TAG}_bench_kernel_stats.csv > gpurun_out/kstats.txt
head -16 gpurun_out/kstats.txt
rm -rf gpurun_out/prof_final
timeout -k 10 900 python bench.py > gpurun_out/bench_full.log 2>&1
tail -1 gpurun_out/bench_full.log > gpurun_out/${TAG}_bench.json
cat gpurun_out/${TAG}_bench.json
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1
tail -1 gpurun_out/bench_driver.log > gpurun_out/${TAG}_bench_driver_form.json
cat gpurun_out/${TAG}_bench_driver_form.json
