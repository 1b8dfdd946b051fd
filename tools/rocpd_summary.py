#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (rocpd SQLite database or *_kernel_trace.csv):
per-kernel calls / mean / total, the GEMM-level family mean (every kernel that runs an
MLP GEMM level: k_gemm, k_fwd*, k_axk16, k_dw_part* + k_dw_fin — a split-K level is one
part + one fin launch), and the gaps between back-to-back dispatches.

usage: python tools/rocpd_summary.py <run_results.db | kernel_trace.csv> [--since-last N]
       --since-last N: only the last N GEMM-level dispatches' time span (the timed windows)
"""
import csv
import glob
import os
import re
import sqlite3
import sys

LEVEL = ("k_gemm<", "k_fwd<", "k_fwd16<", "k_fwd16p<", "k_axk16<", "k_dw_part<", "k_dw_part16")


def load(path):
    if path.endswith(".csv"):
        rows = []
        for r in csv.DictReader(open(path)):
            rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        return sorted(rows, key=lambda x: x[1])
    db = sqlite3.connect(path)
    cur = db.cursor()
    names = [r[0] for r in cur.execute("select name from sqlite_master where type='table'")]
    kd = [n for n in names if n.startswith("rocpd_kernel_dispatch")][0]
    ks = [n for n in names if n.startswith("rocpd_info_kernel_symbol")][0]
    sym = {i: (dn or kn) for i, kn, dn in cur.execute(f"select id, kernel_name, display_name from {ks}")}
    rows = [(sym[k], s, e) for k, s, e in cur.execute(f"select kernel_id, start, end from {kd}")]
    return sorted(rows, key=lambda x: x[1])


def short(name):
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*$", "", name)
    return name.replace("sacmi::", "")


def main(path, since_last=None):
    rows = load(path)
    if since_last:
        idx = [i for i, r in enumerate(rows) if short(r[0]).startswith(LEVEL)]
        first = idx[-since_last] if len(idx) >= since_last else 0
        rows = rows[first:]
    stats = {}
    for n, s, e in rows:
        k = short(n)
        c = stats.setdefault(k, [0, 0])
        c[0] += 1
        c[1] += e - s
    tot = sum(v[1] for v in stats.values())
    for k, (n, t) in sorted(stats.items(), key=lambda kv: -kv[1][1]):
        print(f"{k[:78]:78s} {n:7d} {t / n / 1e3:9.3f} us {100 * t / tot:6.2f}%")
    lv_t = sum(t for k, (n, t) in stats.items() if k.startswith(LEVEL) or k.startswith("k_dw_fin"))
    lv_n = sum(n for k, (n, t) in stats.items() if k.startswith(LEVEL))
    if lv_n:
        print(f"\nGEMM levels: {lv_n} levels, mean {lv_t / lv_n / 1e3:.3f} us per level")
    gaps = [rows[i + 1][1] - rows[i][2] for i in range(len(rows) - 1)]
    small = [g for g in gaps if 0 <= g < 20000]
    if small:
        small.sort()
        print(f"back-to-back gaps (< 20 us): {len(small)}, median {small[len(small) // 2] / 1e3:.3f} us, "
              f"mean {sum(small) / len(small) / 1e3:.3f} us")
    print(f"span {(rows[-1][2] - rows[0][1]) / 1e3:.1f} us, busy {tot / 1e3:.1f} us over {len(rows)} dispatches")


if __name__ == "__main__":
    args = sys.argv[1:]
    n = None
    if "--since-last" in args:
        i = args.index("--since-last")
        n = int(args[i + 1])
        del args[i:i + 2]
    p = args[0] if args else "gpurun_out/prof"
    if os.path.isdir(p):
        c = glob.glob(os.path.join(p, "**", "*.db"), recursive=True) + \
            glob.glob(os.path.join(p, "**", "*kernel_trace.csv"), recursive=True)
        p = c[0]
    main(p, n)
