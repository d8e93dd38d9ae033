set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_intab -o run -- python3 $R/tools/int_ab.py 3 > $R/gpurun_out/r02_int_ab_prof.log 2>&1; echo "prof rc=$?"
cd $R && python tools/kstats.py gpurun_out/prof_intab/run_results.db | grep -i integrate
