#!/bin/bash
# GPU box: A/B digests of the previous and the current libofx build, then the kernel trace of the current one
set -e
mkdir -p gpurun_out
OFX_LIB=tools/ablib/libofx_prev.so timeout -k 10 300 python -u tools/ab_gn.py > gpurun_out/ab_prev.json
timeout -k 10 300 python -u tools/ab_gn.py > gpurun_out/ab_cur.json
cat gpurun_out/ab_prev.json gpurun_out/ab_cur.json
if [ "${AB_PROF:-1}" = 1 ]; then
  R=$(pwd)
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_ab -o run -- python3 $R/bench.py --no-cpu-baseline --steps 20 > $R/gpurun_out/bench_ab.log 2>&1
  cd $R
  python tools/kstats.py gpurun_out/prof_ab/run_results.db > gpurun_out/kstats_ab.txt
  head -20 gpurun_out/kstats_ab.txt
  grep '"metric"' gpurun_out/bench_ab.log | cut -c1-400
fi
