# Schwarz-default lines for configs 1 / 2 / 4 and the moose pair; the refresh-threshold study on the moose
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
timeout -k 10 400 python tools/moose_rot_tol.py || exit $?
for c in 1 2 4; do
  timeout -k 10 400 python bench.py --config $c --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r05s_bench_config$c.log 2>&1 || exit $?
  tail -1 gpurun_out/r05s_bench_config$c.log > gpurun_out/r05_bench_config$c.json
  python -c "import json; d=json.loads(open('gpurun_out/r05_bench_config$c.json').read()); r=d['roofline']; print($c, round(d['value'],1), r['iterations_per_frame'], r['launches_per_frame'])"
done
timeout -k 10 300 python bench.py --moose --steps 20 --warmup 3 > gpurun_out/moose.log 2>&1 || exit $?
tail -1 gpurun_out/moose.log > gpurun_out/r05_moose.json; cat gpurun_out/r05_moose.json
