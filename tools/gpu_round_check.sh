#!/bin/bash
# GPU box: the full -m gpu suite, smoke(), and bench lines of BASELINE configs 1 / 2 / 4 and config 5's scenes of
# ranks 1 and 7 (round-end evidence)
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests/ -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_full.log 2>&1
tail -3 gpurun_out/gputest_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
tail -1 gpurun_out/smoke.log
for c in 1 2 4; do
  timeout -k 10 400 python bench.py --config $c --no-cpu-baseline --steps 30 > gpurun_out/bench_config$c.log 2>&1
  tail -1 gpurun_out/bench_config$c.log | cut -c1-200
done
for r in 1 7; do
  timeout -k 10 400 python bench.py --config 5 --scene-rank $r --no-cpu-baseline --steps 50 > gpurun_out/bench_config5_r$r.log 2>&1
  tail -1 gpurun_out/bench_config5_r$r.log | cut -c1-200
done
