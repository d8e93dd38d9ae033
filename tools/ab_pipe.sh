# A/B on one box: GN loop stream modes (OFX_GN_PIPE = 0 caller stream / 1 two streams / 2 one internal stream /
# 3 two high-priority streams), bench.py 100 frames each, two rounds
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for i in 1 2; do
  for v in 0 1 2 3; do
    OFX_GN_PIPE=$v timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/abp_$v$i.json 2> gpurun_out/abp_$v$i.err
    python -c "import json; d=json.loads(open('gpurun_out/abp_$v$i.json').read().strip().splitlines()[-1]); print('pipe$v', round(d['value'],2), round(d['breakdown_ms']['solve'],3), round(d['roofline']['avg_launch_us'],3))"
  done
done
