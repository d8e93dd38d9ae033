# Round end with a bitwise check: gn_2k / gn_4k chain digests of the current library against a previous build copied to
# ./libofx_base_tmp.so (tools/ab_gn.py; a change meant to keep every bit must match), then tools/round_final.sh
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
