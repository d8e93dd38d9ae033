set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02_gputest0.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 50 --no-cpu-baseline > gpurun_out/r02_bench0.log 2>&1 && \
bash tools/pmc_valu.sh
