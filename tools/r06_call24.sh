set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
ROUNDS=3 bash tools/ab_libs.sh cur noslab
