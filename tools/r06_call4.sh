set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
DIAG_NODES=3 timeout -k 10 120 python tools/one_launch_diag.py gn_4k.npz 0 > gpurun_out/r06c4_diag.log 2>&1; rc=$?; tail -6 gpurun_out/r06c4_diag.log; [ $rc -eq 0 ] || exit $rc
DIAG_NODES=4 timeout -k 10 120 python tools/one_launch_diag.py gn_4k.npz 0 > gpurun_out/r06c4_diag4.log 2>&1; rc=$?; tail -4 gpurun_out/r06c4_diag4.log
