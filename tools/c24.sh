# k_terms: an ARAP edge's weight and node i's records loaded with the edge (two memory trips instead of three): GPU suite,
# digests against the previous library, bench A/B, kernel stats of both
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
R=$(pwd)
timeout -k 10 600 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/ > gpurun_out/c24_suite.log 2>&1; rc=$?
tail -2 gpurun_out/c24_suite.log
if [ $rc -ne 0 ]; then grep -h "FAILED\|Error" gpurun_out/c24_suite.log | head -20; exit $rc; fi
lib() { case $1 in base) echo $R/libofx_base_tmp.so;; *) echo $R/occlusionfusion_amd/libofx.so;; esac; }
for v in base new; do
  OFX_LIB=$(lib $v) timeout -k 10 300 python -u tools/ab_gn.py > gpurun_out/dig_$v.json || exit $?
  echo "$v $(cat gpurun_out/dig_$v.json)" | cut -c1-300
done
for i in 1 2; do
  for v in base new; do
    OFX_LIB=$(lib $v) timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 --warmup 5 > gpurun_out/w_$v$i.json 2> gpurun_out/w_$v$i.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/w_$v$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', round(d['value'],1), round(d['ms_per_step'],4), r.get('iterations_per_frame'), r.get('launches_per_frame'), round(r.get('avg_launch_us'),3))"
  done
done
cd /tmp && export TMPDIR=/tmp
for v in base new; do
  OFX_LIB=$(lib $v) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$v -o run -- python3 $R/bench.py --no-cpu-baseline --steps 20 > $R/gpurun_out/prof_$v.log 2>&1 || exit $?
  python $R/tools/kstats.py $R/gpurun_out/prof_$v/run_results.db > $R/gpurun_out/kstats_$v.txt
  echo "== $v"; grep -h "k_terms\|k_assemble" $R/gpurun_out/kstats_$v.txt
  rm -rf $R/gpurun_out/prof_$v
done
