"""Duration distribution (percentiles, us) of one kernel from a rocprofv3 rocpd SQLite database (tuning tool).

  python tools/kdist.py gpurun_out/prof/run_results.db k_pcg_iter
"""
import sqlite3
import sys

import numpy as np

db, name = sys.argv[1], sys.argv[2]
c = sqlite3.connect(db)
q = """select d.end-d.start from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
       where s.kernel_name like ? order by d.start"""
d = np.array([r[0] for r in c.execute(q, (f"%{name}%",))], dtype=np.float64) / 1e3
print(f"{name}: n={len(d)} mean={d.mean():.2f} us")
print("percentiles 5/25/50/75/95:", np.round(np.percentile(d, [5, 25, 50, 75, 95]), 2))
h, e = np.histogram(d, bins=20, range=(0, 12))
for k in range(len(h)):
    if h[k]:
        print(f"  {e[k]:5.1f}-{e[k + 1]:5.1f} us: {h[k]}")
