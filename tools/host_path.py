#!/usr/bin/env python3
"""Where the drop-in's per-update time goes (diagnostic): the single-update graph on the
device timeline, back-to-back launches, synchronous steps, and the trainer loop's pieces
(select_action, push, the staged rows' flush, update_parameters).
usage: tools/host_path.py [--config 2] [--n 200]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "humanoid-walking-with-sac_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench as B  # noqa: E402


def per_call_us(fn, n):
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return 1e6 * (time.perf_counter() - t0) / n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--n", type=int, default=200)
    a = ap.parse_args()
    args = B.parse_args(["--config", str(a.config)])
    wl = B.workload(args)
    from sac_imp import SAC
    S, A, H, Bt = wl["S"], wl["A"], wl["H"], wl["batch"]
    torch.manual_seed(0)
    agent = SAC(S, A, hidden_dim=H, device="cuda", capacity=100_000, max_batch=Bt, seed=3,
                networks=wl["networks"], compute_dtype=wl["dtype"])
    ctx = agent._ctx
    ctx.push(*B.synth(20_000, 11, S, A))
    for _ in range(20):
        ctx.step(Bt)
    ctx.synchronize()
    print(f"sync ctx.step            {per_call_us(lambda: ctx.step(Bt), a.n):8.1f} us")

    def burst():
        for _ in range(20):
            ctx.step_async(Bt)
        ctx.synchronize()
    burst()
    print(f"step_async x20 + sync    {per_call_us(burst, a.n // 20) / 20:8.1f} us per update")
    t_launch = []
    for _ in range(a.n):
        t0 = time.perf_counter()
        ctx.step_async(Bt)
        t_launch.append(time.perf_counter() - t0)
        ctx.synchronize()
    print(f"step_async host call     {1e6 * np.median(t_launch):8.1f} us (median)")
    ks, graph_us = ctx.profile_timeline(Bt, 1)
    ks = sorted(ks, key=lambda k: k["start_us"])
    print(f"single-update graph      {graph_us:8.1f} us (HIP events around the replay)")
    t_first = ks[0]["start_us"]
    t_end = max(k["end_us"] for k in ks)
    print(f"  first kernel entry at  {t_first:8.1f} us, last exit at {t_end:.1f} us")
    for k in ks:
        print(f"    {k['site']:30s} {k['start_us']:8.1f} {k['end_us'] - k['start_us']:7.2f}")
    # trainer-loop pieces
    rng = np.random.default_rng(12)
    st = rng.standard_normal((a.n + 2, S)).astype(np.float32)
    tt = np.zeros(5)
    per = []
    for i in range(a.n):
        t0 = time.perf_counter()
        act = agent.select_action(st[i])
        t1 = time.perf_counter()
        agent.replay_buffer.push(st[i], act, 0.1, st[i + 1], False)
        t2 = time.perf_counter()
        agent.replay_buffer._flush()
        t3 = time.perf_counter()
        agent.update_parameters(Bt)
        t4 = time.perf_counter()
        tt += [t1 - t0, t2 - t1, t3 - t2, t4 - t3, t4 - t0]
        per.append([t1 - t0, t2 - t1, t3 - t2, t4 - t3])
    tt *= 1e6 / a.n
    per = 1e6 * np.array(per)
    print("trainer loop medians: select %.1f push %.1f flush %.1f update %.1f; update p90 %.1f max %.1f" % (
        *np.median(per, axis=0), np.percentile(per[:, 3], 90), per[:, 3].max()))
    print(f"trainer loop: select_action {tt[0]:.1f}  push {tt[1]:.1f}  flush {tt[2]:.1f}  "
          f"update_parameters {tt[3]:.1f}  total {tt[4]:.1f} us")
    print(f"select_action alone      {per_call_us(lambda: agent.select_action(st[0]), a.n):8.1f} us")

    def act_upd():
        agent.select_action(st[0])
        agent.update_parameters(Bt)

    def push_upd():
        agent.replay_buffer.push(st[0], st[0][:A], 0.1, st[1], False)
        agent.update_parameters(Bt)
    print(f"select_action + update   {per_call_us(act_upd, a.n):8.1f} us")
    print(f"push + update            {per_call_us(push_upd, a.n):8.1f} us")
    print(f"update alone             {per_call_us(lambda: agent.update_parameters(Bt), a.n):8.1f} us")


if __name__ == "__main__":
    main()
