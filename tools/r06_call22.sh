set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -s -m gpu --timeout 200 --timeout-method thread tests/test_gpu_schwarz.py -k "mfma or gn_2k_chain or moose" > gpurun_out/r06c22_tests.log 2>&1; rc=$?
grep -h "PCG\|passed\|failed\|Error\|error" gpurun_out/r06c22_tests.log | head -20
[ $rc -ne 0 ] && exit $rc
OFX_AS_INV_MFMA=1 OFX_LIB=tools/stampslib/libofx_stamps.so timeout -k 10 180 python tools/as_invert_stamps.py > gpurun_out/r06c22_inv1.log 2>&1 || exit $?
tail -9 gpurun_out/r06c22_inv1.log
