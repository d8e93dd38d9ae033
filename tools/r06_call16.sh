set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
OFX_LIB=tools/stampslib/libofx_stamps.so timeout -k 10 180 python tools/as_iter_stamps.py > gpurun_out/r06c16_stamps.log 2>&1 || exit $?
cat gpurun_out/r06c16_stamps.log
