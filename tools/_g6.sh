set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
for v in v2w8 v2w6; do
  export OFX_LIB=$R/tools/variants/libofx_$v.so
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$v -o run -- python3 tools/int_ab.py 3 > $R/gpurun_out/ab_$v.log 2>&1 || { echo "fail $v"; exit 1; }
  timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES --kernel-include-regex 'k_integrate' -f csv -d $R/gpurun_out/pmc_$v -o run -- python3 tools/int_ab.py 3 > $R/gpurun_out/pmc_$v.log 2>&1 || { echo "pmc fail $v"; exit 1; }
  unset OFX_LIB
  python tools/kstats.py gpurun_out/prof_$v/run_results.db | grep -i "integrate"
done
