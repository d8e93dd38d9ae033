# Round end: bitwise digests of the gn_2k / gn_4k chains against the previous library (k_terms' edge loads must not
# change a bit), then tools/round_final.sh (suite, smoke, measurement, configs 2 / 4, moose)
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
R=$(pwd)
for v in base new; do
  L=$R/occlusionfusion_amd/libofx.so; [ $v = base ] && L=$R/libofx_base_tmp.so
  OFX_LIB=$L timeout -k 10 300 python -u tools/ab_gn.py > gpurun_out/dig_$v.json || exit $?
  echo "$v $(cat gpurun_out/dig_$v.json)" | cut -c1-200
done
bash tools/round_final.sh
