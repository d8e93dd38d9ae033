# Per-point k-NN skinning over 16 lanes per point (k_skin_points: the prefetch stream's longest kernel beside the solve):
# GPU suite, bench A/B against the previous library (100 frames each, alternating, three rounds), kernel stats
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 600 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/ > gpurun_out/c21_suite.log 2>&1; rc=$?
tail -2 gpurun_out/c21_suite.log
if [ $rc -ne 0 ]; then grep -h "FAILED\|Error" gpurun_out/c21_suite.log | head -20; exit $rc; fi
lib() { case $1 in base) echo $R/libofx_base_tmp.so;; *) echo $R/occlusionfusion_amd/libofx.so;; esac; }
for i in 1 2 3; do
  for v in base new; do
    OFX_LIB=$(lib $v) timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 --warmup 5 > gpurun_out/s_$v$i.json 2> gpurun_out/s_$v$i.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/s_$v$i.json').read().strip().splitlines()[-1]); r=d['roofline']; ri=d['roofline_integrate']; print('$v', round(d['value'],1), round(d['ms_per_step'],4), round(d['breakdown_ms']['solve'],4), r.get('launches_per_frame'), round(r.get('avg_launch_us'),3), round(ri['in_loop_avg_launch_us'],2))"
  done
done
cd /tmp && export TMPDIR=/tmp
OFX_LIB=$(lib new) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_s -o run -- python3 $R/bench.py --no-cpu-baseline --steps 20 > $R/gpurun_out/prof_s.log 2>&1 || exit $?
python $R/tools/kstats.py $R/gpurun_out/prof_s/run_results.db > $R/gpurun_out/kstats_s.txt
grep -h "k_skin_points\|k_as_apply\|k_pcg_iter" $R/gpurun_out/kstats_s.txt
rm -rf $R/gpurun_out/prof_s
