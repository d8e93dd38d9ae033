#!/bin/bash
# Round 6: the setup scan in one 32k-entry tile (k_scan) — the GN / Schwarz / prefetch suites (bitwise and oracle tests),
# then bench A/B against the previous build (tools/ablib/libofx_old.so), alternating.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_golden_gn.py tests/test_gpu_schwarz.py tests/test_gpu_prefetch.py tests/test_gpu_stoprule.py > gpurun_out/r06_scan_tests.log 2>&1 || { tail -40 gpurun_out/r06_scan_tests.log; exit 1; }
tail -2 gpurun_out/r06_scan_tests.log
ROUNDS=3 timeout -k 10 700 bash tools/ab_libs.sh old cur
