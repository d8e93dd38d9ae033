set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
OFX_LIB=tools/stampslib/libofx_stamps.so timeout -k 10 180 python tools/as_iter_stamps.py > gpurun_out/r06c11_stamps.log 2>&1 || exit $?
head -10 gpurun_out/r06c11_stamps.log | tail -9
timeout -k 10 400 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_schwarz.py > gpurun_out/r06c11_schwarz.log 2>&1 || { tail -30 gpurun_out/r06c11_schwarz.log; exit 1; }
tail -2 gpurun_out/r06c11_schwarz.log
ROUNDS=3 bash tools/ab_libs.sh base cur
