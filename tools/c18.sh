# Integrate occupancy: k_integrate_pal4 at 7 and 8 waves per SIMD (tuning builds -DOFX_INT_WPE=7|8; 72 / 64 VGPRs with
# 12 / 56 bytes of scratch) against the current 6; bench 60 frames per run, alternating, three rounds
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
R=$(pwd)
for i in 1 2 3; do
  for v in cur w7 w8; do
    L=$R/occlusionfusion_amd/libofx.so; [ $v != cur ] && L=$R/libofx_${v}_tmp.so
    OFX_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 60 --warmup 5 > gpurun_out/o_$v$i.json 2> gpurun_out/o_$v$i.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/o_$v$i.json').read().strip().splitlines()[-1]); r=d['roofline_integrate']; print('$v', round(d['value'],1), round(r['avg_launch_us'],2), round(r['in_loop_avg_launch_us'],2), round(r['frac'],4))"
  done
done
