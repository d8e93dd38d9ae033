# k_pcg_w0 with its list and stop flag first and its stores last: GPU suite, digests against the previous library,
# bench A/B (100 frames each, alternating, two rounds), kernel stats of both
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 600 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/ > gpurun_out/c29_suite.log 2>&1; rc=$?
tail -2 gpurun_out/c29_suite.log
if [ $rc -ne 0 ]; then grep -h "FAILED\|Error" gpurun_out/c29_suite.log | head -20; exit $rc; fi
lib() { case $1 in base) echo $R/libofx_base_tmp.so;; *) echo $R/occlusionfusion_amd/libofx.so;; esac; }
for v in base new; do
  OFX_LIB=$(lib $v) timeout -k 10 300 python -u tools/ab_gn.py > gpurun_out/dig_$v.json || exit $?
  echo "$v $(cat gpurun_out/dig_$v.json)" | cut -c1-200
done
for i in 1 2; do
  for v in base new; do
    OFX_LIB=$(lib $v) timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 --warmup 5 > gpurun_out/w_$v$i.json 2> gpurun_out/w_$v$i.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/w_$v$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', round(d['value'],1), round(d['ms_per_step'],4), r.get('launches_per_frame'), round(r.get('avg_launch_us'),3))"
  done
done
cd /tmp && export TMPDIR=/tmp
for v in base new; do
  OFX_LIB=$(lib $v) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$v -o run -- python3 $R/bench.py --no-cpu-baseline --steps 20 > $R/gpurun_out/prof_$v.log 2>&1 || exit $?
  python $R/tools/kstats.py $R/gpurun_out/prof_$v/run_results.db > $R/gpurun_out/kstats_$v.txt
  echo "== $v"; grep -h "k_pcg_w0\|k_pcg_proj2\|k_terms" $R/gpurun_out/kstats_$v.txt
  rm -rf $R/gpurun_out/prof_$v
done
