set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
run() {  # $1 = label, $2 = env assignment or ""
  timeout -k 10 300 env $2 python bench.py --no-cpu-baseline > gpurun_out/ab10_$1.json 2> gpurun_out/ab10_$1.err || { echo "fail $1"; tail -5 gpurun_out/ab10_$1.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/ab10_$1.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$1', round(d['value'],2), r['iterations_per_frame'], r['launches_per_frame'], round(r['avg_launch_us'],3), round(d['roofline_integrate']['avg_launch_us'],1))"
}
for i in 1 2; do
  run base$i "OFX_PCG_STREAM=0"
  run s3_$i "OFX_PCG_STREAM=3"
  run s2_$i "OFX_PCG_STREAM=2"
done
