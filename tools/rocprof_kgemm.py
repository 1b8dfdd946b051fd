#!/usr/bin/env python3
"""Summarise a rocprofv3 --stats kernel CSV: per-kernel mean duration, and the mean
per GEMM level over every kernel that runs a grouped-GEMM level (the bench's roofline
kernel family: every sacmi::k_gemm instantiation, k_fwd / k_fwd16 for the large-M bf16
forward levels, k_axk16 for the bf16 dh levels, k_dw_part / k_dw_part16 + k_dw_fin for the split-K bf16 weight-gradient
levels — one level = one part launch + one fin launch), for the agreement check against
bench.py's `roofline.avg_launch_us`."""
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    tot_ns = calls = 0
    level = ("sacmi::k_gemm<", "sacmi::k_fwd_x6<", "sacmi::k_fwd16<", "sacmi::k_fwd16p<", "sacmi::k_axk16<", "sacmi::k_axk_x6<", "sacmi::k_dw_part")
    for r in rows:
        name, n, avg = r["Name"], int(r["Calls"]), float(r["AverageNs"])
        print(f"{name[:72]:72s} {n:7d} {avg / 1e3:9.2f} us  {float(r['Percentage']):6.2f}%")
        if any(k in name for k in level):
            tot_ns += avg * n
            calls += n
        elif "sacmi::k_dw_fin" in name:
            tot_ns += avg * n                   # second kernel of a split-K level
    if calls:
        print(f"\nGEMM levels (k_gemm all tile configs + k_fwd_x6 / k_fwd16* + k_axk16 / k_axk_x6 + k_dw_part* / k_dw_fin): "
              f"{calls} levels, mean {tot_ns / calls / 1e3:.3f} us")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_stats.csv")
