#!/bin/bash
# VALU / wave-cycle counters of the warped integrate kernel (one PMC pass per counter group).
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_VMEM_RD \
  --kernel-include-regex 'k_integrate|k_pcg_iter' -f csv -d $R/gpurun_out/pmc_valu -o run -- \
  python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/pmc_valu.log 2>&1
