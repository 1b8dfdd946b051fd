#!/usr/bin/env python3
"""Per-kernel VGPR / spill / occupancy table from hipcc -Rpass-analysis=kernel-resource-usage
(development aid).  usage: resources.py file.hip [extra hipcc flags]"""
import re
import subprocess
import sys

cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950",
       "-munsafe-fp-atomics", "-fno-gpu-rdc", "-I/root/repo/include", "-c", sys.argv[1],
       "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:]
err = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in err.split("\n"):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark: +([A-Za-z ]+?)(?: \[[a-z/]+\])?: (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for k, v in rows.items():
    print(f"{k[:95]:95s} vgpr {v.get('VGPRs', '?'):>4} agpr {v.get('AGPRs', '?'):>3} "
          f"spill {v.get('VGPRs Spill', '?'):>3} occ {v.get('Occupancy', '?')} lds {v.get('LDS Size', '?')}")
