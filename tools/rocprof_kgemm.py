#!/usr/bin/env python3
"""Summarise a rocprofv3 --stats kernel CSV: per-kernel mean duration, and the mean
over every sacmi::k_gemm instantiation (the bench's roofline kernel), for the
agreement check against bench.py's `roofline.avg_launch_us`."""
import csv
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    tot_ns = calls = 0
    for r in rows:
        name, n, avg = r["Name"], int(r["Calls"]), float(r["AverageNs"])
        print(f"{name[:72]:72s} {n:7d} {avg / 1e3:9.2f} us  {float(r['Percentage']):6.2f}%")
        if "sacmi::k_gemm<" in name:
            tot_ns += avg * n
            calls += n
    if calls:
        print(f"\nsacmi::k_gemm (all tile configs): {calls} launches, mean {tot_ns / calls / 1e3:.3f} us")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_stats.csv")
