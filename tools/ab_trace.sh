#!/bin/bash
# A/B of libofx builds by traced kernel durations (tuning, not product): for each library (tools/ablib/libofx_<tag>.so,
# or "cur" for the in-tree build), alternating over ROUNDS, a kernel-traced short bench; prints the traced average of
# the PCG iteration and the per-GN-step kernels plus the bench line's frames/s and launch time.
#   bash tools/ab_trace.sh base cur        (ROUNDS=2 STEPS=20 by default)
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for r in $(seq 1 ${ROUNDS:-2}); do
  for L in "$@"; do
    P=$R/tools/ablib/libofx_$L.so; [ "$L" = cur ] && P=$R/occlusionfusion_amd/libofx.so
    export OFX_LIB=$P
    (cd /tmp && TMPDIR=/tmp timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/abt -o run -- \
      python3 $R/bench.py --no-cpu-baseline --steps ${STEPS:-20} > $R/gpurun_out/abt.log 2>&1)
    python3 - "$L" <<'EOF'
import json, sqlite3, sys, glob
db = glob.glob("gpurun_out/abt/**/run_results.db", recursive=True) or glob.glob("gpurun_out/abt/run_results.db")
c = sqlite3.connect(db[0])
q = """select s.kernel_name, count(*), avg(d.end-d.start) from rocpd_kernel_dispatch d
       join rocpd_info_kernel_symbol s on d.kernel_id = s.id group by s.kernel_name"""
rows = {n: (k, a / 1e3) for n, k, a in c.execute(q)}
def pick(key):
    m = [(k, a) for n, (k, a) in rows.items() if key in n]
    if not m: return "-"
    k = sum(x[0] for x in m); return f"{sum(x[0] * x[1] for x in m) / k:.2f}"
line = [l for l in open("gpurun_out/abt.log") if l.startswith("{")][-1]
d = json.loads(line)
print(sys.argv[1], "fps", round(d["value"], 1), "launch_us", round(d["roofline"]["avg_launch_us"], 3),
      "| traced us: iter", pick("k_pcg_iter"), "assemble", pick("k_assemble"), "terms", pick("k_terms"),
      "proj", pick("k_pcg_projILb"), "proj2", pick("k_pcg_proj2"), "w0", pick("k_pcg_w0"), flush=True)
EOF
    rm -rf $R/gpurun_out/abt
  done
done
