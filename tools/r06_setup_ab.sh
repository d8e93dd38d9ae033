#!/bin/bash
# Round 6: setup kernels (k_scan in one tile; k_pair_count / k_pair_scatter with every load ahead of the atomics) —
# the GN / Schwarz / prefetch / stop-rule suites, per-kernel traced times of the setup kernels for the previous build
# (tools/ablib/libofx_old.so) and this one, then the bench A/B, alternating.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_golden_gn.py tests/test_gpu_schwarz.py tests/test_gpu_prefetch.py tests/test_gpu_stoprule.py tests/test_gpu_moose.py > gpurun_out/r06_setup_tests.log 2>&1 || { tail -40 gpurun_out/r06_setup_tests.log; exit 1; }
tail -2 gpurun_out/r06_setup_tests.log
for L in old cur; do
  P=$R/tools/ablib/libofx_$L.so; [ "$L" = cur ] && P=$R/occlusionfusion_amd/libofx.so
  (cd /tmp && export TMPDIR=/tmp && OFX_LIB=$P timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/setup_$L -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 20 --warmup 2 > $R/gpurun_out/setup_$L.log 2>&1) || { tail -20 gpurun_out/setup_$L.log; exit 1; }
  f=$(find gpurun_out/setup_$L -name "*kernel_stats.csv" | head -1)
  echo "lib $L"; grep -E "k_scan|k_pair_count|k_pair_scatter|k_seg_rank|k_as_tab" "$f" | cut -d, -f1-5
done
ROUNDS=3 timeout -k 10 700 bash tools/ab_libs.sh old cur
