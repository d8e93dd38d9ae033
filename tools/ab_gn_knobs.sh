# In-box A/B: k_as_apply's lanes per segment (OFX_AS_LANES 2 / 4) and a 3-solution warm start (tuning build
# libofx_kp3_tmp.so), bench 100 frames each, alternating
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
OFX_AS_LANES=4 timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_schwarz.py 2>&1 | tail -2 || exit $?
for i in 1 2 3; do
  for v in l2 l4 kp3; do
    E="OFX_NONE=1"; [ $v = l4 ] && E="OFX_AS_LANES=4"; [ $v = kp3 ] && E="OFX_LIB=$PWD/libofx_kp3_tmp.so"
    env $E timeout -k 10 300 python bench.py --no-cpu-baseline --steps 100 --warmup 5 > gpurun_out/k_$v$i.json 2> gpurun_out/k_$v$i.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/k_$v$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', round(d['value'],1), round(d['ms_per_step'],4), r.get('iterations_per_frame'), r.get('launches_per_frame'), round(r.get('avg_launch_us'),3))"
  done
done
