#!/bin/bash
# Issue / wait split of the bench's kernels (one PMC pass, <= 8 SQ counters): VALU instructions and busy
# quad-cycles vs wave cycles parked in s_waitcnt / barriers (SQ_WAIT_ANY) — the evidence for "VALU-bound"
# (integrate) and "latency-bound" (k_pcg_iter, k_assemble, k_terms) in DESIGN.md §5.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_INSTS_SALU \
  --kernel-include-regex 'k_integrate|k_pcg_iter|k_as_iter|k_as_w0|k_as_proj2|k_as_invert|k_as_apply|k_assemble|k_terms' -f csv -d $R/gpurun_out/pmc_valu -o run -- \
  python3 $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/gpurun_out/pmc_valu.log 2>&1
