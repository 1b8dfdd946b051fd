#!/usr/bin/env python3
"""Per-kernel body / gap split of one update on the launch timeline (diagnostic).

Runs the bench workload's context (config, networks, dtype), captures `n` updates with
sacmi_profile_timeline and prints, per launch site averaged over the updates: the body
(first-workgroup entry -> last-workgroups exit) and the gap to the next kernel's entry.
usage: tools/timeline_dump.py [--config 2] [--n 20] [--fill 200000]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "humanoid-walking-with-sac_amd"))

import bench as B  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--n", type=int, default=20)
    ap.add_argument("--fill", type=int, default=200_000)
    ap.add_argument("--networks", default="model1")
    a = ap.parse_args()
    args = B.parse_args(["--config", str(a.config), "--networks", a.networks])
    wl = B.workload(args)
    from sacmi import Config, Context
    ctx = Context(Config(wl["S"], wl["A"], wl["H"], max_batch=args.batch, capacity=a.fill, seed=1,
                         replay=wl["replay"], n_hidden=wl["n_hidden"], compute_dtype=wl["dtype"]), 0)
    B.init_agent(ctx, 0)
    for c0 in range(0, a.fill, 100_000):
        ctx.push(*B.synth(min(100_000, a.fill - c0), 1000 + c0, wl["S"], wl["A"]))
    ctx.step_many_async(args.batch, a.n)
    ctx.synchronize()
    ks, graph_us = ctx.profile_timeline(args.batch, a.n)
    ks = sorted(ks, key=lambda k: k["start_us"])
    side = [k for k in ks if k["site"].endswith("_next")]     # side stream: overlaps the chain
    ks = [k for k in ks if not k["site"].endswith("_next")]
    acc = {}
    for k in side:
        e = acc.setdefault((k["site"], k["kernel"], k["grid"]), [0.0, 0.0, 0])
        e[0] += k["end_us"] - k["start_us"]
        e[2] += 1
    for i, k in enumerate(ks):
        nxt = ks[i + 1]["start_us"] if i + 1 < len(ks) else k["end_us"]
        e = acc.setdefault((k["site"], k["kernel"], k["grid"]), [0.0, 0.0, 0])
        e[0] += k["end_us"] - k["start_us"]
        e[1] += nxt - k["end_us"]
        e[2] += 1
    print(f"graph {graph_us / a.n:.2f} us per update ({a.n} updates)")
    print(f"{'site':34s} {'kernel':12s} {'grid':>5s} {'n':>3s} {'body':>7s} {'gap':>6s}")
    tb = tg = 0.0
    for (site, kern, grid), (b, g, n) in acc.items():
        print(f"{site:34s} {kern:12s} {grid:5d} {n:3d} {b / n:7.2f} {g / n:6.2f}")
        if not site.endswith("_next"):
            tb += b
            tg += g
    print(f"per update: body {tb / a.n:.2f} gap {tg / a.n:.2f}")


if __name__ == "__main__":
    main()
