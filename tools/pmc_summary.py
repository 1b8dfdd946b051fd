#!/usr/bin/env python3
"""HBM-side traffic per GEMM level from two rocprofv3 --pmc passes (tools/gpu_pmc.sh):
FETCH_SIZE and WRITE_SIZE, both in KB per dispatch.  A level is one sacmi::k_gemm,
k_fwd / k_fwd16 or k_axk16 launch, or one split-K k_dw_part* launch plus its k_dw_fin
(bench.py's roofline counts launches the same way).

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
        key = "sacmi::k_gemm" if name.startswith("void sacmi::k_gemm<") else name.split("(")[0]
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
    # the GEMM-level family: per level = all their bytes / the number of levels
    lv = [k for k in rows if k.startswith(("sacmi::k_gemm", "void sacmi::k_fwd", "void sacmi::k_axk16",
                                           "sacmi::k_dw_part", "void sacmi::k_dw_part"))]
    fin = [k for k in rows if "k_dw_fin" in k]
    n_lv = sum(rows[k]["launches"] for k in lv)
    per_level = None
    if n_lv:
        tot = lambda f: sum(rows[k][f] * rows[k]["launches"] for k in lv + fin)
        per_level = {"launches": n_lv, "fetch_bytes": tot("fetch_bytes") / n_lv,
                     "write_bytes": tot("write_bytes") / n_lv, "traffic_bytes": tot("traffic_bytes") / n_lv}
    res = {"kernel": "GEMM levels (k_gemm, k_fwd*, k_axk16, k_dw_part* + k_dw_fin)",
           "per_launch": per_level,
           "correction": "FETCH_SIZE x2 (gfx950 wide-read half count); KB -> bytes x1024",
           "all": rows}
    if out:
        json.dump(res, open(out, "w"), indent=1)
    return res


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out", sys.argv[2] if len(sys.argv) > 2 else None)
