#!/usr/bin/env python3
"""Per-kernel cache counters from the two rocprofv3 --pmc passes of tools/gpu_pmc_cache.sh.

* L2 hit rate = TCC_HIT / (TCC_HIT + TCC_MISS) (MI355X_MICROARCH.md, L2 section), per
  kernel and over the GEMM levels (pmc_summary.LEVEL).  TCC_REQ counts every L2 request
  (reads, writes, atomics); TCC_EA0_RDREQ the L2's read requests to the fabric (MALL /
  HBM), reported as counted (the gfx950 FETCH_SIZE half-count note applies to bytes, not
  to this ratio).
* L1: TCP_TCC_READ_REQ = the L1's read requests to L2 (L1 misses incl. uncached reads),
  TCP_TOTAL_CACHE_ACCESSES its cache accesses; the mean L1 -> L2 read latency in cycles =
  TCP_TCC_READ_REQ_LATENCY / TCP_TCC_READ_REQ.
Counts are per dispatch (summed over the chip's instances of each block).

usage: pmc_cache_summary.py <pass dir> <out.json> [bench args]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import LEVEL, counters, csrc_digest  # noqa: E402

P1 = ("TCC_HIT", "TCC_MISS", "TCC_REQ", "TCC_EA0_RDREQ")
P2 = ("TCP_TCC_READ_REQ", "TCP_TOTAL_CACHE_ACCESSES", "TCP_TCC_READ_REQ_LATENCY", "TCP_PENDING_STALL_CYCLES")


def per_dispatch(p, k, c):
    v = p.get(k, {})
    for name in (c, c + "_sum"):
        if name in v:
            return v[name][0] / max(v[name][1], 1)
    return 0.0


def main(root, out, args=""):
    p = [counters(os.path.join(root, f"p{i}")) for i in (1, 2)]
    kernels = sorted(set(p[0]) | set(p[1]))
    rows = {}
    for k in kernels:
        r = {"launches": max(p[0].get(k, {}).get("duration_ns", [0, 0])[1],
                             p[1].get(k, {}).get("duration_ns", [0, 0])[1]),
             "duration_ns": per_dispatch(p[0], k, "duration_ns")}
        for c in P1:
            r[c] = per_dispatch(p[0], k, c)
        for c in P2:
            r[c] = per_dispatch(p[1], k, c)
        hm = r["TCC_HIT"] + r["TCC_MISS"]
        r["l2_hit_rate"] = r["TCC_HIT"] / hm if hm else None
        r["l1_l2_latency_cycles"] = (r["TCP_TCC_READ_REQ_LATENCY"] / r["TCP_TCC_READ_REQ"]
                                     if r["TCP_TCC_READ_REQ"] else None)
        rows[k] = r
    lv = [k for k in rows if k.startswith(LEVEL)]
    n = sum(rows[k]["launches"] for k in lv)
    agg = None
    if n:
        tot = lambda key: sum(rows[k][key] * rows[k]["launches"] for k in lv) / n
        agg = {c: tot(c) for c in P1 + P2 + ("duration_ns",)}
        agg["levels"] = n
        agg["l2_hit_rate"] = agg["TCC_HIT"] / (agg["TCC_HIT"] + agg["TCC_MISS"])
        agg["l1_l2_latency_cycles"] = agg["TCP_TCC_READ_REQ_LATENCY"] / max(agg["TCP_TCC_READ_REQ"], 1)
    print(f"{'kernel':58s} {'n':>6s} {'us':>7s} {'L2hit':>6s} {'TCC_REQ':>9s} {'EA_RD':>9s} "
          f"{'L1->L2':>9s} {'L1acc':>9s} {'lat':>6s}")
    for k, v in sorted(rows.items(), key=lambda kv: -kv[1]["launches"]):
        hr = v["l2_hit_rate"]
        lat = v["l1_l2_latency_cycles"]
        print(f"{k[:58]:58s} {v['launches']:6d} {v['duration_ns'] / 1e3:7.2f} "
              f"{hr if hr is not None else float('nan'):6.3f} {v['TCC_REQ']:9.0f} {v['TCC_EA0_RDREQ']:9.0f} "
              f"{v['TCP_TCC_READ_REQ']:9.0f} {v['TCP_TOTAL_CACHE_ACCESSES']:9.0f} "
              f"{lat if lat is not None else float('nan'):6.0f}")
    res = {"kernel": "GEMM levels (pmc_summary.LEVEL)", "bench_args": args, "csrc_digest": csrc_digest(),
           "per_level": agg, "kernels": rows,
           "note": "counts per dispatch, summed over the chip's block instances; L2 hit rate = "
                   "TCC_HIT / (TCC_HIT + TCC_MISS); latency = TCP_TCC_READ_REQ_LATENCY / TCP_TCC_READ_REQ"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(agg))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "")
