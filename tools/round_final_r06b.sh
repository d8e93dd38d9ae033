# Part B of the round-6 end check: the bench line (with the CPU baseline) and the driver's form, configs 1 / 2 / 4, config 5's scenes of ranks 1 and 7, the moose line (outputs under
# gpurun_out/, copied into profiles/ afterwards; every GPU step has its own limit; stops at the first failure).
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
export TAG=r06
timeout -k 10 900 python bench.py > gpurun_out/bench_full.log 2>&1 || { tail -20 gpurun_out/bench_full.log; exit 1; }
tail -1 gpurun_out/bench_full.log > gpurun_out/r06_bench.json
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver.log 2>&1 || { tail -20 gpurun_out/bench_driver.log; exit 1; }
tail -1 gpurun_out/bench_driver.log > gpurun_out/r06_bench_driver_form.json
for c in 1 2 4; do
  timeout -k 10 400 python bench.py --config $c --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r06s_bench_config$c.log 2>&1 || exit $?
  tail -1 gpurun_out/r06s_bench_config$c.log > gpurun_out/r06_bench_config$c.json
done
for r in 1 7; do
  timeout -k 10 400 python bench.py --config 5 --scene-rank $r --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/r06s_bench_config5_r$r.log 2>&1 || exit $?
  tail -1 gpurun_out/r06s_bench_config5_r$r.log > gpurun_out/r06_bench_config5_r$r.json
done
timeout -k 10 300 python bench.py --moose --steps 20 --warmup 3 > gpurun_out/moose.log 2>&1 || exit $?
tail -1 gpurun_out/moose.log > gpurun_out/r06_moose.json
for f in r06_bench r06_bench_driver_form r06_bench_config1 r06_bench_config2 r06_bench_config4 r06_bench_config5_r1 r06_bench_config5_r7; do python -c "import json; d=json.loads(open('gpurun_out/$f.json').read()); r=d['roofline']; print('$f', round(d['value'],1), r['iterations_per_frame'], r['launches_per_frame'], round(r['avg_launch_us'],3), round(r['frac'],3))"; done
python -c "import json; d=json.loads(open('gpurun_out/r06_moose.json').read()); print('moose', d['value'], d['default']['pcg_iterations'], d['default']['max_abs_err_vs_f64_oracle'])"
head -24 gpurun_out/kstats.txt
