#!/usr/bin/env python3
"""Per-GEMM-level counters from the three rocprofv3 --pmc passes of tools/gpu_pmc.sh.

A level is one sacmi::k_gemm, k_fwd / k_fwd16 or k_axk16 launch, or one split-K k_dw_part*
launch plus its k_dw_fin (bench.py's roofline counts levels the same way).

* traffic = FETCH_SIZE x 2 + WRITE_SIZE per level (bytes past L2).  gfx950 correction
  (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports exactly half of the bytes of a
  wide coalesced streaming read -> doubled.  WRITE_SIZE is exact for 16-B-per-lane stores;
  4-B-per-lane epilogue stores are uncalibrated, reported as measured.  The counters are
  L2 memory-side requests: Infinity-Cache hits are included (an upper bound on HBM bytes).
* mfma_busy = sum SQ_VALU_MFMA_BUSY_CYCLES / (sum dispatch duration x 2.4 GHz x 1024 SIMDs)
  over the level kernels: the fraction of the levels' wall time the MFMA pipes of all
  SIMDs were busy (dispatch durations from the same counter pass).  mfma_busy_gui is
  rocprofv3's MfmaUtil form, normalised by GRBM_GUI_ACTIVE / 8 XCDs instead, which reads
  high on short dispatches (MI355X_MICROARCH.md, DVFS note) and so reads low here.
  mfma_flops = SQ_INSTS_VALU_MFMA_MOPS_* x 512.
* csrc_digest: hash of the kernel sources the counters were taken on; bench.py uses the
  file only while the sources are unchanged.

usage: pmc_summary.py <pass dir> <out.json> [bench args]
"""
import csv
import glob
import hashlib
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LEVEL = ("k_gemm<", "k_fwd_x6<", "k_fwd16<", "k_fwd16p<", "k_axk16<", "k_axk_x6<", "k_dw_part16", "k_dw_part_x6")


def csrc_digest(root=ROOT):
    h = hashlib.sha256()
    src = os.path.join(root, "humanoid-walking-with-sac_amd", "csrc")
    for f in sorted(os.listdir(src)):
        if f.endswith((".hip", ".h")):
            h.update(f.encode())
            h.update(open(os.path.join(src, f), "rb").read())
    return h.hexdigest()[:16]


def short(name):
    name = name.split("(")[0]
    for p in ("void ", "sacmi::"):
        name = name.replace(p, "")
    return name


def counters(pass_dir):
    """{kernel: {counter: [sum, dispatches]}} from one pass's counter_collection.csv"""
    acc = defaultdict(lambda: defaultdict(lambda: [0.0, 0]))
    files = glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True)
    seen = set()
    for f in files:
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            c = acc[k][r["Counter_Name"]]
            c[0] += float(r["Counter_Value"])
            key = (r.get("Dispatch_Id"), r["Counter_Name"])
            if key not in seen:
                seen.add(key)
                c[1] += 1
            if (r.get("Dispatch_Id"), "dur") not in seen:
                seen.add((r.get("Dispatch_Id"), "dur"))
                d = acc[k]["duration_ns"]
                d[0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                d[1] += 1
    return acc


def main(root, out, args=""):
    p = [counters(os.path.join(root, f"p{i}")) for i in (1, 2, 3)]
    kernels = sorted(set(p[0]) | set(p[1]) | set(p[2]))
    rows = {}
    for k in kernels:
        f = p[0].get(k, {}).get("FETCH_SIZE", [0, 0])
        w = p[1].get(k, {}).get("WRITE_SIZE", [0, 0])
        m = p[2].get(k, {})
        n = max(f[1], w[1], 1)
        rows[k] = {"launches": n, "fetch_bytes": 2 * f[0] * 1024 / max(f[1], 1),
                   "write_bytes": w[0] * 1024 / max(w[1], 1),
                   "mfma_busy_cycles": m.get("SQ_VALU_MFMA_BUSY_CYCLES", [0, 1])[0] / max(m.get("SQ_VALU_MFMA_BUSY_CYCLES", [0, 1])[1], 1),
                   "gui_active": m.get("GRBM_GUI_ACTIVE", [0, 1])[0] / max(m.get("GRBM_GUI_ACTIVE", [0, 1])[1], 1),
                   "duration_ns": m.get("duration_ns", [0, 1])[0] / max(m.get("duration_ns", [0, 1])[1], 1),
                   "mfma_flops": 512 * (m.get("SQ_INSTS_VALU_MFMA_MOPS_F32", [0, 1])[0] +
                                        m.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", [0, 1])[0]) /
                                 max(m.get("SQ_INSTS_VALU_MFMA_MOPS_F32", [0, 1])[1], 1)}
        rows[k]["traffic_bytes"] = rows[k]["fetch_bytes"] + rows[k]["write_bytes"]
    lv = [k for k in rows if k.startswith(LEVEL)]
    fin = [k for k in rows if k.startswith("k_dw_fin")]
    n_lv = sum(rows[k]["launches"] for k in lv)
    per_level = None
    if n_lv:
        tot = lambda key, ks: sum(rows[k][key] * rows[k]["launches"] for k in ks)
        busy = tot("mfma_busy_cycles", lv + fin)
        gui = tot("gui_active", lv + fin)
        dur = tot("duration_ns", lv + fin)
        per_level = {"levels": n_lv,
                     "fetch_bytes": tot("fetch_bytes", lv + fin) / n_lv,
                     "write_bytes": tot("write_bytes", lv + fin) / n_lv,
                     "traffic_bytes": tot("traffic_bytes", lv + fin) / n_lv,
                     "mfma_flops": tot("mfma_flops", lv + fin) / n_lv,
                     "duration_ns_under_pmc": dur / n_lv,
                     "mfma_busy": busy / (dur * 2.4 * 1024) if dur else None,
                     "mfma_busy_gui": busy / (gui / 8 * 1024) if gui else None}
    for k, v in sorted(rows.items(), key=lambda kv: -kv[1]["launches"]):
        u = v["mfma_busy_cycles"] / (v["duration_ns"] * 2.4 * 1024) if v["duration_ns"] else 0
        print(f"{k[:58]:58s} {v['launches']:6d} fetch {v['fetch_bytes'] / 1e6:8.3f} MB write "
              f"{v['write_bytes'] / 1e6:7.3f} MB  mfma {v['mfma_flops'] / 1e9:7.3f} GF busy {u:6.3f}")
    res = {"kernel": "GEMM levels (k_gemm, k_fwd*, k_axk16, k_dw_part* + k_dw_fin)",
           "bench_args": args, "csrc_digest": csrc_digest(), "per_level": per_level,
           "correction": "FETCH_SIZE x2 (gfx950 wide-read half count); KB -> bytes x1024; "
                         "GRBM_GUI_ACTIVE / 8 (summed over the XCDs), 1024 SIMDs",
           "kernels": rows}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(per_level))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "")
