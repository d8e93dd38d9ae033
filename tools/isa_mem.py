"""Compressed memory-op / wait / branch sequence of one kernel in a gfx950 .s file (tuning tool).

  hipcc ... --cuda-device-only -S gn.hip -o /tmp/gn.s && python tools/isa_mem.py /tmp/gn.s <mangled-name>
"""
import re
import sys

s = open(sys.argv[1]).read()
i = s.index(sys.argv[2] + ':')
j = s.index('s_endpgm', i)
body = s[i:j].split('\n')
out, prev, cnt = [], None, 0
for l in body:
    t = l.strip()
    m = re.match(r'(global_load\w*|global_store\w*|s_load\w*|s_waitcnt[^;]*|s_cbranch\w*|ds_\w+|s_barrier|scratch\w*|\.LBB\w+:)', t)
    if m:
        k = m.group(1)
        if k == prev:
            cnt += 1
            continue
        if prev:
            out.append(f"{prev} x{cnt}")
        prev, cnt = k, 1
if prev:
    out.append(f"{prev} x{cnt}")
print(len(body), "lines")
print("\n".join(out))
