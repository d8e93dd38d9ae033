set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
TAG=r05 timeout -k 10 1400 bash tools/measure_round.sh > gpurun_out/measure.log 2>&1; rc=$?; tail -5 gpurun_out/measure.log | cut -c1-400
exit $rc
