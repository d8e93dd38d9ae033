set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_integrate_cull.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c7_tests.log 2>&1; rc=$?; tail -2 gpurun_out/c7_tests.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python tools/cull_ab.py --reps 30 > gpurun_out/c7_cullab.log 2>&1 || exit $?
tail -1 gpurun_out/c7_cullab.log
cd /tmp && export TMPDIR=/tmp && cd ${GRAFT_REPO_ROOT}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c7_prof -o run -- python3 tools/cull_ab.py --reps 20 > gpurun_out/c7_prof.log 2>&1 || exit $?
