# Cluster-block configs after the per-step chain / k_terms / skinning changes: config 2 (30 frames) and the moose
# optimize with the library of the first round-5 measurement (def1d26) against the current one, alternating, two rounds
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
R=$(pwd)
for i in 1 2; do
  for v in old new; do
    L=$R/occlusionfusion_amd/libofx.so; [ $v = old ] && L=$R/libofx_old_tmp.so
    OFX_LIB=$L timeout -k 10 300 python bench.py --config 2 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/c2_$v$i.json 2> gpurun_out/c2_$v$i.err || exit $?
    OFX_LIB=$L timeout -k 10 300 python bench.py --moose --steps 20 --warmup 3 > gpurun_out/mo_$v$i.json 2> gpurun_out/mo_$v$i.err || exit $?
    python -c "
import json
d=json.loads(open('gpurun_out/c2_$v$i.json').read().strip().splitlines()[-1]); m=json.loads(open('gpurun_out/mo_$v$i.json').read().strip().splitlines()[-1])
print('$v', 'config2', round(d['value'],1), round(d['roofline']['avg_launch_us'],3), 'moose_ms', round(m['value'],3), m['default']['pcg_iterations'])"
  done
done
