set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/c8_prof -o run -- python3 $R/bench.py --no-cpu-baseline --steps 20 --warmup 5 > $R/gpurun_out/c8_bench.log 2>&1 || exit $?
cd $R
python tools/gap_timeline.py gpurun_out/c8_prof/run_kernel_trace.csv > gpurun_out/c8_gaps.txt 2>&1; cat gpurun_out/c8_gaps.txt | head -40
