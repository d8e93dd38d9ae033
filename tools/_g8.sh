set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r02_gputest5.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r02_gputest5.log
[ $rc -le 1 ] || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ab8 -o run -- python3 $R/tools/int_ab.py 3 > $R/gpurun_out/ab8.log 2>&1; echo "ab rc=$?"
cd $R
python tools/kstats.py gpurun_out/prof_ab8/run_results.db | grep -i integrate
timeout -k 10 400 python bench.py --gpus 2 --backend gloo --mode shard --solve replicated --steps 20 --no-cpu-baseline > gpurun_out/shard2_repl.log 2>&1; echo "shard repl rc=$?"
timeout -k 10 400 python bench.py --gpus 2 --backend gloo --mode shard --solve allreduce --steps 20 --no-cpu-baseline > gpurun_out/shard2_ar.log 2>&1; echo "shard ar rc=$?"
