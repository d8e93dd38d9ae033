# A/B: Schwarz rings of 12 (product) against 16 (tuning build libofx_r16_tmp.so): fixture parity, then the bench
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
OFX_LIB=$PWD/libofx_r16_tmp.so timeout -k 10 400 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gpu_schwarz.py 2>&1 | grep -h "Schwarz:\|Schwarz \|passed\|failed" || exit $?
for i in 1 2; do
  for v in r12 r16; do
    E="OFX_NONE=1"; [ $v = r16 ] && E="OFX_LIB=$PWD/libofx_r16_tmp.so"
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 --warmup 5 > gpurun_out/rg_$v$i.json 2> gpurun_out/rg_$v$i.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/rg_$v$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', round(d['value'],1), round(d['ms_per_step'],4), r.get('iterations_per_frame'), r.get('launches_per_frame'), round(r.get('avg_launch_us'),3), r['preconditioner']['segments'])"
  done
done
