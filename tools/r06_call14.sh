set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_schwarz.py tests/test_gpu_stoprule.py tests/test_gpu_moose.py > gpurun_out/r06c14_tests.log 2>&1 || { tail -40 gpurun_out/r06c14_tests.log; exit 1; }
tail -1 gpurun_out/r06c14_tests.log
ROUNDS=3 bash tools/ab_libs.sh w0 cur
