#!/usr/bin/env python3
"""HBM-side traffic per sacmi::k_gemm launch from two rocprofv3 --pmc passes
(tools/gpu_pmc.sh): FETCH_SIZE and WRITE_SIZE, both in KB per dispatch.

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports exactly half
of the bytes of a wide coalesced streaming read -> doubled here.  WRITE_SIZE is exact for
16-B-per-lane stores; our epilogues store 4 B per lane (uncalibrated width), so the write
figure is reported as measured.  These counters are L2 memory-side requests: Infinity
Cache hits are included, so `traffic` is "bytes past L2", an upper bound on HBM bytes.

usage: pmc_summary.py gpurun_out [out.json]
"""
import csv
import json
import os
import sys
from collections import defaultdict


def per_kernel(path, counter):
    acc = defaultdict(lambda: [0.0, 0])
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        key = "sacmi::k_gemm" if name.startswith("void sacmi::k_gemm<") else name
        acc[key][0] += float(r["Counter_Value"])
        acc[key][1] += 1
    return {k: (v[0] / v[1], v[1]) for k, v in acc.items()}


def main(root, out=None):
    f = per_kernel(os.path.join(root, "pmc_FETCH_SIZE", "run_counter_collection.csv"), "FETCH_SIZE")
    w = per_kernel(os.path.join(root, "pmc_WRITE_SIZE", "run_counter_collection.csv"), "WRITE_SIZE")
    rows = {}
    for k in sorted(set(f) | set(w)):
        if not k.startswith(("sacmi", "void sacmi")):
            continue
        fk, n = f.get(k, (0.0, 0))
        wk, _ = w.get(k, (0.0, 0))
        rows[k] = {"launches": n, "fetch_bytes": 2 * fk * 1024, "write_bytes": wk * 1024,
                   "traffic_bytes": 2 * fk * 1024 + wk * 1024}
    for k, v in rows.items():
        print(f"{k[:60]:60s} {v['launches']:6d}  fetch {v['fetch_bytes'] / 1e6:8.3f} MB  "
              f"write {v['write_bytes'] / 1e6:8.3f} MB")
    res = {"kernel": "sacmi::k_gemm", "per_launch": rows.get("sacmi::k_gemm"),
           "correction": "FETCH_SIZE x2 (gfx950 wide-read half count); KB -> bytes x1024",
           "all": rows}
    if out:
        json.dump(res, open(out, "w"), indent=1)
    return res


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out", sys.argv[2] if len(sys.argv) > 2 else None)
