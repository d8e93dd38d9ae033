# Part A of the round-6 end check of the default tree: the GPU suite, smoke, measure_round.sh (PMC traffic, VALU split,
# kernel stats, the bench line and the driver form). Outputs under gpurun_out/ (copied into profiles/ afterwards). Every
# GPU step has its own limit; stops at the first failure.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
export TAG=r06
timeout -k 10 600 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/ > gpurun_out/r06_gputest_final.txt 2>&1; rc=$?
tail -3 gpurun_out/r06_gputest_final.txt
if [ $rc -ne 0 ]; then grep -h "FAILED\|Error" gpurun_out/r06_gputest_final.txt | head -20; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
bash tools/measure_round.sh > gpurun_out/final_measure.log 2>&1 || { tail -30 gpurun_out/final_measure.log; exit 1; }
head -24 gpurun_out/kstats.txt
