# Kernel-trace profile of the default bench (20 frames): per-kernel stats and the GPU idle-gap timeline
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv rocpd -d $R/gpurun_out/c27_prof -o run -- python3 $R/bench.py --no-cpu-baseline --steps 20 --warmup 5 > $R/gpurun_out/c27_bench.log 2>&1 || exit $?
cd $R
python tools/kstats.py gpurun_out/c27_prof/run_results.db > gpurun_out/c27_kstats.txt 2>&1; head -24 gpurun_out/c27_kstats.txt
python tools/gap_timeline.py gpurun_out/c27_prof/run_kernel_trace.csv 20 > gpurun_out/c27_gaps.txt 2>&1; head -40 gpurun_out/c27_gaps.txt
