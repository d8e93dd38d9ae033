set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
OFX_LIB=tools/stampslib/libofx_stamps.so timeout -k 10 180 python tools/as_invert_stamps.py > gpurun_out/r06c21_inv1.log 2>&1 || exit $?
OFX_AS_INV_MFMA=0 OFX_LIB=tools/stampslib/libofx_stamps.so timeout -k 10 180 python tools/as_invert_stamps.py > gpurun_out/r06c21_inv0.log 2>&1 || exit $?
tail -9 gpurun_out/r06c21_inv1.log; tail -8 gpurun_out/r06c21_inv0.log
