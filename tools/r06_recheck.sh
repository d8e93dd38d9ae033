#!/bin/bash
# Round-6 re-entry check of the committed tree: the GPU suite, smoke(), one default bench line (no CPU leg).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06b_gputest.log 2>&1 || { tail -30 gpurun_out/r06b_gputest.log; exit 1; }
tail -3 gpurun_out/r06b_gputest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06b_smoke.log 2>&1 || { tail -20 gpurun_out/r06b_smoke.log; exit 1; }
tail -1 gpurun_out/r06b_smoke.log
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r06b_bench.log 2>&1 || { tail -20 gpurun_out/r06b_bench.log; exit 1; }
tail -1 gpurun_out/r06b_bench.log | cut -c1-400
