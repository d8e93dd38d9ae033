# Integrate: branch-free trip loads (tuning build -DOFX_INT_UNCOND) against the current library: the integrate GPU tests
# on the variant, then bench 60 frames per run, alternating, three rounds (roofline_integrate: isolated and in-loop)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
R=$(pwd)
OFX_LIB=$R/libofx_unc_tmp.so timeout -k 10 600 python -u -m pytest -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_integrate_edges.py tests/test_gpu_integrate_cull.py tests/test_gpu_configs.py tests/test_gpu_full.py tests/test_gpu_parity.py > gpurun_out/c17_suite.log 2>&1; rc=$?
tail -2 gpurun_out/c17_suite.log
if [ $rc -ne 0 ]; then grep -h "FAILED\|Error" gpurun_out/c17_suite.log | head -20; exit $rc; fi
for i in 1 2 3; do
  for v in cur unc; do
    L=$R/occlusionfusion_amd/libofx.so; [ $v = unc ] && L=$R/libofx_unc_tmp.so
    OFX_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 60 --warmup 5 > gpurun_out/i_$v$i.json 2> gpurun_out/i_$v$i.err || exit $?
    python -c "import json; d=json.loads(open('gpurun_out/i_$v$i.json').read().strip().splitlines()[-1]); r=d['roofline_integrate']; print('$v', round(d['value'],1), round(r['avg_launch_us'],2), round(r['in_loop_avg_launch_us'],2), round(r['frac'],4))"
  done
done
