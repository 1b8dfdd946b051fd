#!/usr/bin/env python3
"""Compact view of a kernel's load / vmcnt-wait / MFMA sequence from a hipcc --save-temps .s
(development aid): L = vector-memory load, S = store, W<n> = s_waitcnt vmcnt(n),
M<k> = k consecutive MFMAs, | = branch/label.
usage: isa_loads.py file.s mangled_kernel_name"""
import re
import sys

src, name = sys.argv[1], sys.argv[2]
lines = open(src).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith(name + ":"))
out, m = [], 0
for l in lines[start + 1:]:
    if "s_endpgm" in l:
        break
    t = l.strip()
    tok = None
    if t.startswith("v_mfma"):
        m += 1
        continue
    if m:
        out.append(f"M{m}")
        m = 0
    if re.match(r"(global|buffer)_load", t):
        tok = "L"
    elif re.match(r"(global|buffer)_store", t):
        tok = "S"
    elif t.startswith("s_waitcnt") and "vmcnt" in t:
        tok = "W" + re.search(r"vmcnt\((\d+)\)", t).group(1)
    elif t.startswith("s_cbranch") or t.startswith(".LBB"):
        tok = "|"
    if tok:
        if tok == "|" and out and out[-1] == "|":
            continue
        out.append(tok)
print(" ".join(out))
