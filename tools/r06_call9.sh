set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
R=$(pwd)
mkdir -p gpurun_out
bash tools/pmc_traffic.sh && python tools/pmc_summary.py gpurun_out gpurun_out/r06_pmc_traffic.json && cat gpurun_out/r06_pmc_traffic.json | head -40
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex 'k_as_iter|k_pcg_iter|k_as_apply' -f csv -d $R/gpurun_out/pmc_tcc6 -o run -- python3 $R/bench.py --no-cpu-baseline --steps 4 --warmup 1 > $R/gpurun_out/pmc_tcc6.log 2>&1
cd $R
python - <<'PY'
import csv, glob, collections
rows = []
for f in glob.glob("gpurun_out/pmc_tcc6/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in d.items()}, len(next(iter(d.values()))))
PY
