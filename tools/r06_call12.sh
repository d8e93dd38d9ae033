set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_schwarz.py -k one_launch > gpurun_out/r06c12_schwarz.log 2>&1 || { tail -30 gpurun_out/r06c12_schwarz.log; exit 1; }
tail -1 gpurun_out/r06c12_schwarz.log
OFX_LIB=tools/stampslib/libofx_stamps.so timeout -k 10 180 python tools/as_iter_stamps.py > gpurun_out/r06c12_stamps.log 2>&1 || exit $?
head -10 gpurun_out/r06c12_stamps.log | tail -8
ROUNDS=3 bash tools/ab_libs.sh cur0 cur1 cur
