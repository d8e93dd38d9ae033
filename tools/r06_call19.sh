set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
STEPS=100 VAR=OFX_PCG_RATIO ROUNDS=4 bash tools/ab_env.sh 2 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/prof19 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 10 --warmup 3 > $R/gpurun_out/r06c19_rocprof.log 2>&1
cd $R
python tools/rocclr_in_loop.py gpurun_out/prof19/run_results.db --warmup 3 --steps 10 > gpurun_out/r06c19_glue.txt
rm -rf gpurun_out/prof19
cat gpurun_out/r06c19_glue.txt
