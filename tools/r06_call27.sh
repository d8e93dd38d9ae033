set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 300 python tools/host_probe.py > gpurun_out/r06c27_host.log 2>&1 || { tail -20 gpurun_out/r06c27_host.log; exit 1; }
head -45 gpurun_out/r06c27_host.log
