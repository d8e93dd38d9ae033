# Schwarz apply: the slab rows issued right after the stop test, ahead of the gathers (tuning build -DOFX_AS_SLAB_T1),
# against the current library: gn_2k / gn_4k digests, bench 100 frames each (alternating, three rounds), traced apply
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
R=$(pwd)
lib() { case $1 in slab) echo $R/libofx_slab_tmp.so;; *) echo $R/occlusionfusion_amd/libofx.so;; esac; }
for v in cur slab; do
  OFX_LIB=$(lib $v) timeout -k 10 300 python -u tools/ab_gn.py > gpurun_out/dig_$v.json || exit $?
  echo "$v $(cat gpurun_out/dig_$v.json)" | cut -c1-200
done
for i in 1 2 3; do
  for v in cur slab; do
    OFX_LIB=$(lib $v) timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 --warmup 5 > gpurun_out/a_$v$i.json 2> gpurun_out/a_$v$i.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/a_$v$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', round(d['value'],1), round(d['ms_per_step'],4), round(d['breakdown_ms']['solve'],4), r.get('launches_per_frame'), round(r.get('avg_launch_us'),3))"
  done
done
cd /tmp && export TMPDIR=/tmp
for v in cur slab; do
  OFX_LIB=$(lib $v) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$v -o run -- python3 $R/bench.py --no-cpu-baseline --steps 20 > $R/gpurun_out/prof_$v.log 2>&1 || exit $?
  python $R/tools/kstats.py $R/gpurun_out/prof_$v/run_results.db > $R/gpurun_out/kstats_$v.txt
  echo "== $v"; grep -h "k_as_apply\|k_pcg_iter" $R/gpurun_out/kstats_$v.txt
  rm -rf $R/gpurun_out/prof_$v
done
