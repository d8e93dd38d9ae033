set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 120 python tools/one_launch_diag.py gn_4k.npz 5 > gpurun_out/r06c3_diag4k.log 2>&1; rc=$?; cat gpurun_out/r06c3_diag4k.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/one_launch_diag.py gn_2k.npz 3 OFX_PCG_W1=1 > gpurun_out/r06c3_diag2k_w1.log 2>&1; rc=$?; tail -5 gpurun_out/r06c3_diag2k_w1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/one_launch_diag.py gn_2k.npz 3 OFX_PCG_KU=4 > gpurun_out/r06c3_diag2k_ku4.log 2>&1; rc=$?; tail -5 gpurun_out/r06c3_diag2k_ku4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/one_launch_diag.py gn_1k.npz 3 > gpurun_out/r06c3_diag1k.log 2>&1; rc=$?; tail -5 gpurun_out/r06c3_diag1k.log
