set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum --kernel-include-regex 'k_pcg_iter|k_integrate_pal4|k_assemble' -f csv -d $R/gpurun_out/pmc_tcc -o run -- python3 $R/bench.py --no-cpu-baseline --steps 4 --warmup 1 > $R/gpurun_out/pmc_tcc.log 2>&1 || exit $?
cd $R
python - <<'PY'
import csv, collections, numpy as np
rows=list(csv.DictReader(open('gpurun_out/pmc_tcc/run_counter_collection.csv')))
agg=collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    k=r['Kernel_Name'].split('(')[0][-40:]
    agg[k][r['Counter_Name']].append(float(r['Counter_Value']))
for k,v in agg.items():
    print(k, {c: (round(float(np.median(x))), len(x)) for c,x in v.items()})
PY
