#!/bin/bash
# GPU box: kernel-trace stats of a short bench run with the library $1 (a tuning build) -> gpurun_out/kstats_$2.txt
set -e
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
OFX_LIB=$R/$1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$2 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 20 > $R/gpurun_out/bench_$2.log 2>&1
cd $R
python tools/kstats.py gpurun_out/prof_$2/run_results.db > gpurun_out/kstats_$2.txt
head -24 gpurun_out/kstats_$2.txt
