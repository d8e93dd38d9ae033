#!/bin/bash
# HBM traffic of the bench's two roofline kernels and the GN assembly pair from rocprofv3 PMC counters, one counter per pass
# (FETCH_SIZE and WRITE_SIZE cannot share a TCC pass on gfx950). Output: gpurun_out/pmc_{fetch,write}/.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-include-regex 'k_pcg_iter|k_as_iter|k_as_w0|k_as_proj2|k_as_apply|k_as_invert|k_pcg_proj|k_integrate|k_assemble|k_terms|k_brick_cull|k_tile_max' -f csv \
    -d $R/gpurun_out/pmc_$c -o run -- python3 $R/bench.py --no-cpu-baseline --steps 4 --warmup 1 \
    > $R/gpurun_out/pmc_$c.log 2>&1
done
