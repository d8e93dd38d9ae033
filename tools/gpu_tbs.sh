# GPU round trip used while tuning: gpu tests, phase stamps, 3 bench runs, one kernel-trace profile
timeout -k 10 500 python -m pytest tests -m gpu -x -q > gpurun_out/t.log 2>&1; tail -3 gpurun_out/t.log
OFX_LIB=tools/bin/libofx_stamps.so timeout -k 10 300 python tools/pcg_stamps.py > gpurun_out/st.log 2>&1; grep -v amdgpu.ids gpurun_out/st.log | head -12
for i in 1 2 3; do timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/b$i.log 2>&1 || exit 1; done
for i in 1 2 3; do python -c "import json,sys; d=json.loads(open(\"gpurun_out/b$i.log\").read().strip().splitlines()[-1]); print(round(d[\"value\"],1), {k: round(v,3) for k,v in d[\"breakdown_ms\"].items()}, round(d[\"roofline\"][\"avg_launch_us\"],2), round(d[\"roofline\"][\"launches_per_frame\"],1), round(d[\"roofline_integrate\"][\"avg_launch_us\"],1))"; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/profx -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bp.log 2>&1
python tools/kdist.py gpurun_out/profx/run_results.db k_pcg_iter | head -2
