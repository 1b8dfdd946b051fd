#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy table from hipcc's resource remarks.

usage: python tools/kernel_resources.py csrc/kernels.hip [more .hip]   (run from the package dir)
"""
import re
import subprocess
import sys

FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-fno-gpu-rdc", "-c", "-o", "/dev/null",
         "-Rpass-analysis=kernel-resource-usage"]


def table(src):
    out = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, src], capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
        if m and cur is not None:
            cur[m.group(1).split()[0]] = int(m.group(2))
    return rows


if __name__ == "__main__":
    for src in sys.argv[1:]:
        for r in table(src):
            name = subprocess.run(["c++filt"], input=r["name"], capture_output=True, text=True).stdout.strip()
            name = re.sub(r"\(.*", "", name)
            print(f"{r.get('VGPRs', 0):4d} v {r.get('AGPRs', 0):3d} a {r.get('ScratchSize', 0):4d} scr "
                  f"occ {r.get('Occupancy', 0)} lds {r.get('LDS', 0):6d}  {name}")
