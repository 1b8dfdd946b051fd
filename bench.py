#!/usr/bin/env python3
"""Benchmark: SAC gradient-steps/s on Humanoid-v5 shapes (BASELINE.json `metric`).

One "step" = one full SAC update (sac_imp.py:74-152): device random.sample over the
HBM replay ring (1M rows by default), gather, target, twin-critic fwd/bwd + Adam,
actor fwd/bwd + Adam, alpha update, Polyak — on synthetic Humanoid-shaped data
(obs 376, act 17, hidden 512, batch 256 per GPU; random-init weights).

Single GPU:   python bench.py [--steps K --warmup W]
N GPUs:       python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
              (data parallel: per-GPU replay shard, per-GPU batch 256, critic and actor
              gradients all-reduced over RCCL; value = N * iterations/s, i.e.
              batch-256-equivalent gradient steps per second, weak scaling).

Prints ONE JSON line (rank 0).  Extra objects: `roofline` (dominant kernel = the
grouped fp32 MFMA GEMM, timed with HIP events on its launch stream) and
`cpu_baseline` (the oracle's torch-CPU port of the reference update + deque replay
on this host's cores, bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "humanoid-walking-with-sac_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

S_DIM, A_DIM, HIDDEN, BATCH = 376, 17, 512, 256
PEAK_FP32_MFMA_TFLOPS = 157.3     # MI355X_MICROARCH.md: Peak FP32 (matrix), dense
PEAK_BF16_MFMA_TFLOPS = 2500.0    # MI355X_MICROARCH.md: Peak BF16 MFMA, dense (no sparsity)
PEAK_HBM_GBS = 8000.0

# BASELINE.json configs (index + 1) that run on one GPU / per rank: the shape of the
# networks, the per-GPU batch, the replay kind and the GEMM arithmetic
CONFIGS = {
    2: dict(S=376, A=17, H=512, batch=256, replay="uniform", dtype="fp32",
            workload="BASELINE configs[1]: Humanoid-v5 shapes, hidden=512, batch=256, uniform "
                     "replay (HBM ring, device random.sample)"),
    3: dict(S=376, A=17, H=512, batch=4096, replay="per", dtype="fp32",
            workload="BASELINE configs[2]: Humanoid-v5 shapes, hidden=512, batch=4096, prioritized "
                     "replay resident in HBM (device np.random.choice over prios**alpha); fp32 "
                     "GEMM levels on bf16 MFMA with each fp32 operand split exactly into three "
                     "bf16 parts (6 cross products, fp32 accumulation: the x6 form, DESIGN §13j) "
                     "except the policy heads and the sample backward (fp32 MFMA)"),
    5: dict(S=661, A=23, H=512, batch=4096, replay="uniform", dtype="bf16",
            workload="BASELINE configs[4] per GPU: NAO-walk shapes (obs 661, act 23), hidden=512, "
                     "batch=4096, uniform replay, auto-entropy on, bf16 MFMA operands (fp32 "
                     "accumulation, fp32 master weights / Adam)"),
}


def workload(args) -> dict:
    w = dict(CONFIGS[args.config])
    w["batch"] = args.batch
    if args.dtype:
        w["dtype"] = args.dtype
    w["n_hidden"] = 3 if args.networks == "model2" else 2
    w["networks"] = args.networks
    return w


def necessary_flops(S, A, H, B, n_hidden=2):
    """GEMM FLOPs the update needs (excludes the reference's wasted
    actor-pass Q dW and state columns of Q-fc1 dX); n_hidden-1 H x H layers per net."""
    HH = (n_hidden - 1) * H * H
    Qf = (S + A) * H + HH + H
    Pf = S * H + HH + 2 * H * A
    Qdx = H + HH + H * A
    Pbw = Pf + HH + 2 * H * A
    return 2 * B * ((Pf + 2 * Qf) + 2 * (2 * Qf + H + HH) + (Pf + 2 * Qf + 2 * Qdx + Pbw))


def synth(n, seed, S=S_DIM, A=A_DIM):
    rng = np.random.default_rng(seed)
    s = rng.standard_normal((n, S), dtype=np.float32)
    s2 = rng.standard_normal((n, S), dtype=np.float32)
    a = rng.uniform(-0.4, 0.4, size=(n, A)).astype(np.float32)
    r = rng.standard_normal(n, dtype=np.float32)
    d = (rng.random(n) < 0.02).astype(np.uint8)
    return s, a, r, s2, d


def init_agent(ctx, seed):
    """Xavier-uniform weights, zero biases (networks_model1.py:22-25,60-63; the same for
    networks_model2's critics — its orthogonal policy init changes nothing measured)."""
    rng = np.random.default_rng(seed)
    from sacmi.core import net_keys
    cfg = ctx.cfg
    S, A, H, nh = cfg.state_dim, cfg.action_dim, cfg.hidden_dim, cfg.n_hidden
    shapes = {"policy": {"fc1": (H, S), "mean": (A, H), "log_std": (A, H)},
              "q": {"fc1": (H, S + A), f"fc{nh + 1}": (1, H)}}
    for i in range(2, nh + 1):
        shapes["policy"][f"fc{i}"] = shapes["q"][f"fc{i}"] = (H, H)
    q_sd = {}
    for net in ("policy", "q1", "q2"):
        shp = shapes["policy" if net == "policy" else "q"]
        sd = {}
        for key, _layer, part in net_keys(net, nh):
            lname = key.split(".")[0]
            o, i = shp[lname]
            if part == 0:
                b = np.sqrt(6.0 / (o + i))
                sd[key] = rng.uniform(-b, b, size=(o, i)).astype(np.float32)
            else:
                sd[key] = np.zeros(o, np.float32)
        ctx.set_net(net, sd)
        q_sd[net] = sd
    ctx.set_net("q1_target", q_sd["q1"])
    ctx.set_net("q2_target", q_sd["q2"])


# kernels that run the MLP GEMM levels (the dominant kernel family of the update); L10
# (k_gemm_sample_bwd: dL/da + the sampling backward) and the heads kernel are not levels
LEVEL_KERNELS = {"k_gemm", "k_fwd_x6", "k_fwd16", "k_fwd16p", "k_axk16", "k_axk_x6", "k_dw_part16", "k_dw_part_x6", "k_dw_fin"}


def timeline_roofline(ctx, batch, n_updates, data_parallel=False):
    """Roofline of the GEMM levels measured on the REAL update: the same n-update graph
    the timed windows replay, instrumented so that every kernel stamps its first
    workgroup's entry on the GPU clock (sacmi_profile_timeline), replayed once warm and
    once measured, with HIP events on the context stream around the measured replay.
    Kernels run back to back in the graph, so a launch's duration is the distance to the
    next launch's start (the last: its own end); their sum must equal the event time.
    data_parallel: the sequence of the data-parallel update (sacmi_profile_timeline_dp,
    every rank calls), whose RCCL all-reduces stamp nothing: a kernel followed by one
    ends at its own exit stamp, and the gap up to the next kernel is all-reduce time."""
    ks, graph_us = ctx.profile_timeline(batch, n_updates, data_parallel)
    ks = sorted(ks, key=lambda k: k["start_us"])
    # the next update's sampling + gather on the side stream ("*_next" sites, batch-4096
    # class and prioritized replay) overlap the chain: their own span, outside the chain
    side = [k for k in ks if k["site"].endswith("_next")]
    for k in side:
        k["dur_us"] = k["end_us"] - k["start_us"]
    ks = [k for k in ks if not k["site"].endswith("_next")]
    allreduce_us = 0.0
    for i, k in enumerate(ks):
        nxt = ks[i + 1] if i + 1 < len(ks) else None
        if nxt is None:
            k["dur_us"] = k["end_us"] - k["start_us"]
        elif data_parallel and nxt["site_idx"] > k["site_idx"] + 1:
            k["dur_us"] = k["end_us"] - k["start_us"]
            allreduce_us += nxt["start_us"] - k["end_us"]
        else:
            k["dur_us"] = nxt["start_us"] - k["start_us"]
    lv = [k for k in ks if k["kernel"] in LEVEL_KERNELS]
    gemm_us = sum(k["dur_us"] for k in lv)
    gemm_flops = sum(k["flops"] for k in lv)
    gemm_bytes = sum(k["bytes"] for k in lv)
    levels = sum(1 for k in lv if k["flops"] > 0)          # a split-K pair is one level
    kernel_launches = {}
    for k in lv:
        kernel_launches[k["kernel"]] = kernel_launches.get(k["kernel"], 0) + 1
    sites = {}
    for k in ks:
        e = sites.setdefault(k["site"], [0.0, 0])
        e[0] += k["dur_us"]
        e[1] += 1 if k["flops"] > 0 or k["kernel"] not in LEVEL_KERNELS else 0
    for k in side:
        e = sites.setdefault(k["site"], [0.0, 0])
        e[0] += k["dur_us"]
        e[1] += 1
    return dict(graph_us=graph_us, sum_us=sum(k["dur_us"] for k in ks) + allreduce_us,
                allreduce_us=allreduce_us, n_updates=n_updates,
                gemm_us=gemm_us, gemm_flops=gemm_flops, gemm_bytes=gemm_bytes, levels=levels,
                kernel_launches=kernel_launches,
                achieved_tflops=gemm_flops / (gemm_us * 1e-6) / 1e12,
                sites_us={n: round(t / max(c, 1), 2) for n, (t, c) in sites.items()})


def pmc_counters(config, networks="model1"):
    """Per-GEMM-level PMC figures of this workload (tools/gpu_pmc.sh + tools/pmc_summary.py:
    bytes past L2 from separate FETCH_SIZE / WRITE_SIZE passes, MFMA busy fraction from
    SQ_VALU_MFMA_BUSY_CYCLES / GRBM_GUI_ACTIVE), read from the committed summary ONLY while
    the kernel sources are the ones it was measured on (csrc digest); else None."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from pmc_summary import csrc_digest
    suffix = "" if networks == "model1" else f"_{networks}"
    path = os.path.join(ROOT, "profiles", f"pmc_c{config}{suffix}.json")
    try:
        z = json.load(open(path))
    except (OSError, ValueError):
        return None
    if z.get("csrc_digest") != csrc_digest() or not z.get("per_level"):
        return None
    z["source"] = os.path.relpath(path, ROOT)
    return z


def cpu_threads() -> int:
    """Host threads for the CPU baseline: the CPU share the GPU box grants one GPU
    (OMP_NUM_THREADS, 16 there), never more than the cores present."""
    share = int(os.environ.get("OMP_NUM_THREADS") or 16)
    return max(1, min(share, os.cpu_count() or 1))


def median_windows(fn, windows):
    """[fn() for each window] and their median."""
    vals = [fn() for _ in range(windows)]
    return float(np.median(vals)), vals


def cpu_baseline(rows, seconds=20.0, warmup=5, batch=BATCH, per=False, n_hidden=2, windows=5):
    """The reference update on CPU (oracle torch port, fp32) + the reference's replay
    data path (deque + random.sample, or the prioritized buffer's numpy sampler), timed
    on this host's cores for a bounded number of steps."""
    import random
    from oracle.replay_ref import DequeReplay, PerReplayNumpy
    from oracle.sac_step import OracleSAC, SacConfig, init_params
    threads = cpu_threads()
    torch.set_num_threads(threads)
    s, a, r, s2, d = rows
    S, A = s.shape[1], a.shape[1]
    cfg = SacConfig(S, A, HIDDEN, n_hidden=n_hidden)
    agent = OracleSAC(cfg, init_params(cfg, 0), dtype=torch.float32)
    if per:
        buf = PerReplayNumpy(capacity=len(r))
        buf.fill(rows)
    else:
        buf = DequeReplay(capacity=len(r))
        for i in range(len(r)):
            buf.push(s[i], a[i], float(r[i]), s2[i], bool(d[i]))
    random.seed(0)
    np.random.seed(0)
    gen = torch.Generator().manual_seed(0)

    def one():
        bs, ba, br, bs2, bd = buf.sample(batch)[:5]
        e1 = torch.randn(batch, A, generator=gen).numpy()
        e2 = torch.randn(batch, A, generator=gen).numpy()
        agent.step(bs, ba, br, bs2, bd, e1, e2)

    for _ in range(warmup):
        one()
    counts = []

    def window():
        n = 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds / windows:
            one()
            n += 1
        dt = time.perf_counter() - t0
        counts.append(n)
        return n / dt

    value, rates = median_windows(window, windows)
    cpu = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    replay = ("PrioritizedReplayBuffer numpy sampler (np.random.choice over prios**alpha)"
              if per else "deque/random.sample replay")
    return dict(value=value, unit="grad-steps/s", cores=threads, kind="port",
                windows=[round(x, 2) for x in rates],
                sample=f"median of {windows} windows of {seconds / windows:.1f}s ({sum(counts)} updates "
                       f"after {warmup} warm-up) at batch {batch}; oracle torch-CPU fp32 port of "
                       f"sac_imp.update_parameters + {replay} over {len(r)} rows (float32 rows); "
                       f"{threads} threads (the box's CPU share per GPU) on {cpu}")


def trainer_loop(wl, steps=300, warmup=30, fill=20_000, sync_python_random=False):
    """The reference trainer's inner loop without the environment (trainer.py:182-205):
    per env step select_action(state) -> replay_buffer.push(transition) ->
    update_parameters(batch) (losses synced, as .item() in sac_imp.py:140-144), through
    the drop-in SAC (sac_imp module name).  Returns env-steps/s and the split.
    sync_python_random=True: the reference-faithful index stream — every update also
    advances Python's `random` exactly as the reference's random.sample does
    (replay_buffer.py:15, sac_imp.py:77), the device drawing the same indices."""
    import random
    from sac_imp import SAC
    S, A, H, B = wl["S"], wl["A"], wl["H"], wl["batch"]
    torch.manual_seed(0)
    random.seed(5)
    agent = SAC(S, A, hidden_dim=H, device="cuda", capacity=max(fill * 2, 100_000),
                max_batch=B, seed=3, networks=wl["networks"], compute_dtype=wl["dtype"],
                sync_python_random=sync_python_random)
    agent._ctx.push(*synth(fill, 11, S, A))
    rng = np.random.default_rng(12)
    states = rng.standard_normal((steps + warmup + 1, S)).astype(np.float32)

    def one(i, t):
        a = agent.select_action(states[i])
        t1 = time.perf_counter()
        agent.replay_buffer.push(states[i], a, float(i % 7) * 0.1, states[i + 1], (i % 50) == 49)
        t2 = time.perf_counter()
        agent.update_parameters(B)
        t3 = time.perf_counter()
        t[0] += t1 - t0_[0]; t[1] += t2 - t1; t[2] += t3 - t2
        t0_[0] = t3

    t0_ = [time.perf_counter()]
    tw = [0.0, 0.0, 0.0]
    for i in range(warmup):
        one(i, tw)
    torch.cuda.synchronize()
    tt = [0.0, 0.0, 0.0]
    t0 = time.perf_counter()
    t0_[0] = t0
    for i in range(warmup, warmup + steps):
        one(i, tt)
    dt = time.perf_counter() - t0
    return {"env_steps_per_s": round(steps / dt, 2),
            "us_select_action": round(1e6 * tt[0] / steps, 1),
            "us_push": round(1e6 * tt[1] / steps, 1),
            "us_update_parameters": round(1e6 * tt[2] / steps, 1),
            "sync_python_random": sync_python_random,
            "note": "trainer.py:182-205 loop minus env.step: select_action + push + "
                    f"update_parameters({B}) per env step, drop-in SAC, {fill}-row replay"
                    + ("; Python's random stream advanced as the reference's (faithful indices)"
                       if sync_python_random else "; device index stream (default)")}


def roofline_object(ctx, args, wl, peak, data_parallel=False, step_us_real=None):
    """The line's `roofline` object: the GEMM levels of the real multi-update graph
    (data_parallel: of the data-parallel update sequence, all-reduces included).
    step_us_real: the timed (uninstrumented) graph's time per update; the stamps of the
    instrumented replay (a clock read and a store per workgroup) stretch it by ~1-4 %, and
    the levels' durations are scaled back by that ratio (reported: instrumentation_scale)."""
    upl = max(1, min(args.updates_per_launch, 256))
    info = timeline_roofline(ctx, args.batch, upl, data_parallel)
    raw_tf = info["achieved_tflops"]
    scale = 1.0
    if step_us_real and info["sum_us"] > 0:
        scale = min(1.0, step_us_real / (info["sum_us"] / upl))
        info["gemm_us"] *= scale
        info["achieved_tflops"] = info["gemm_flops"] / (info["gemm_us"] * 1e-6) / 1e12
    # the committed PMC figures were collected on the single-GPU graph (fused Adam levels)
    pmc = None if data_parallel else pmc_counters(args.config, args.networks)
    lvl = pmc["per_level"] if pmc else {}
    per_level_flops = info["gemm_flops"] / max(info["levels"], 1)
    avg_level_us = info["gemm_us"] / max(info["levels"], 1)
    return {"bound": "mfma", "achieved": round(info["achieved_tflops"], 3), "peak": peak,
            "unit": "TFLOP/s", "frac": round(info["achieved_tflops"] / peak, 4),
            "traffic": round(lvl["traffic_bytes"]) if lvl else None,
            "traffic_unit": "bytes past L2 per GEMM level (PMC FETCH_SIZE x2 + WRITE_SIZE)",
            "mfma_busy": round(lvl["mfma_busy"], 4) if lvl and lvl.get("mfma_busy") else None,
            "pmc_source": pmc["source"] if pmc else None,
            "algorithmic_bytes_per_launch": round(info["gemm_bytes"] / max(info["levels"], 1)),
            "kernel": "GEMM levels of the update: " + ", ".join(
                f"sacmi::{k} x{n}" for k, n in sorted(info["kernel_launches"].items())) +
                      f" per {upl} updates ({wl['dtype']} MFMA)",
            "method": ("launch timeline of the data-parallel update sequence (phases + RCCL "
                       "all-reduces, sacmi_profile_timeline_dp, all ranks)" if data_parallel else
                       "launch timeline of the timed multi-update graph (per-kernel GPU-clock "
                       "stamps, sacmi_profile_timeline)") +
                      "; HIP events on the context stream around the same replay",
            "levels_per_step": round(info["levels"] / upl, 2),
            "avg_launch_us": round(avg_level_us, 3),
            "flops_per_launch": round(per_level_flops),
            "gemm_us_per_step": round(info["gemm_us"] / upl, 2),
            "instrumentation_scale": round(scale, 4),
            "achieved_timeline_raw": round(raw_tf, 3),
            "gemm_flops_per_step": round(info["gemm_flops"] / upl),
            "step_us_timeline": round(info["sum_us"] / upl, 2),
            "step_us_hip_events": round(info["graph_us"] / upl, 2),
            "allreduce_us_per_step": round(info["allreduce_us"] / upl, 2) if data_parallel else None,
            "sites_us": info["sites_us"]}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS),
                    help="BASELINE.json configs[1] (2: batch 256 uniform), configs[2] "
                         "(3: batch 4096, prioritized replay in HBM) or configs[4] per GPU "
                         "(5: NAO shapes, batch 4096, bf16 MFMA)")
    ap.add_argument("--networks", default="model1", choices=("model1", "model2"),
                    help="networks_model1 (2 hidden layers) or networks_model2 (3)")
    ap.add_argument("--dtype", default=None, choices=("fp32", "bf16"),
                    help="GEMM operand arithmetic (default: the config's)")
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--fill", type=int, default=1_000_000)
    ap.add_argument("--windows", type=int, default=0,
                    help="timed windows of --steps updates each (median reported); 0: enough "
                         "windows for >= 2000 timed updates (at least 5)")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--updates-per-launch", type=int, default=20,
                    help="updates per device launch (trainer.py updates_per_step loop)")
    ap.add_argument("--force-dp", action="store_true",
                    help="run the data-parallel path even at world size 1 (overhead check)")
    ap.add_argument("--dp-sim-world", type=int, default=0,
                    help="with --force-dp: one GPU runs rank 0's data-parallel sequence of a "
                         "W-rank job through the loopback hook in its one-rank timing mode "
                         "(SACMI_DP_LOOPBACK_ONE_RANK: the sharded Adam on rank 0's chunk, the "
                         "collectives returning the rank's own gradient, no stand-in kernels): "
                         "that rank's work minus the collectives")
    ap.add_argument("--dp-native", action="store_true",
                    help="(default) data parallel through sacmi_step_dp: the library issues "
                         "the RCCL all-reduces inside its own captured graph")
    ap.add_argument("--dp-torch", action="store_true",
                    help="data parallel through torch.distributed all-reduces around the "
                         "library's phase graphs (eager)")
    ap.add_argument("--no-trainer-loop", action="store_true",
                    help="skip the env-free trainer-loop measurement (select_action + push + "
                         "update_parameters per env step)")
    ap.add_argument("--profile-only", action="store_true",
                    help="just run warmup+steps (for rocprofv3 runs)")
    args = ap.parse_args(argv)
    if args.batch is None:                 # both the single-GPU and the DP paths use it
        args.batch = CONFIGS[args.config]["batch"]
    if args.windows <= 0:
        args.windows = min(200, max(5, -(-2000 // max(1, args.steps))))
    return args


def graph_sizes(steps, per_launch):
    """Updates per launch of every launch the timed loop of `steps` updates makes."""
    full, rem = divmod(steps, per_launch)
    return sorted({n for n in ((per_launch if full else 0), rem) if n > 0})


_RESULT_FD = None   # the process's original stdout while fd 1 is routed to stderr


def quiet_stdout() -> None:
    """Route fd 1 to stderr for the rest of the run (RCCL prints a version banner on
    stdout at communicator creation, on every rank): the one JSON result line goes to
    the original stdout through emit()."""
    global _RESULT_FD
    if _RESULT_FD is None:
        sys.stdout.flush()
        _RESULT_FD = os.dup(1)
        os.dup2(2, 1)


def emit(line: str) -> None:
    sys.stdout.flush()
    if _RESULT_FD is None:
        print(line, flush=True)
    else:
        os.write(_RESULT_FD, (line + "\n").encode())


def main():
    args = parse_args()
    quiet_stdout()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    wl = workload(args)
    per = wl["replay"] == "per"
    S, A, H = wl["S"], wl["A"], wl["H"]
    if world > 1 or args.force_dp:
        from sacmi.dp import run_dp_bench
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29531")
        return run_dp_bench(args, rank, world, local_rank, emit)

    from sacmi import Config, Context
    from sacmi import _lib as L
    torch.cuda.init()
    fill = args.fill
    ctx = Context(Config(S, A, H, max_batch=args.batch, capacity=fill, seed=1,
                         replay=wl["replay"], n_hidden=wl["n_hidden"],
                         compute_dtype=wl["dtype"]), 0)
    init_agent(ctx, 0)
    t_fill = time.perf_counter()
    chunk = 100_000
    rows_keep = None
    for c0 in range(0, fill, chunk):
        rows = synth(min(chunk, fill - c0), 1000 + c0, S, A)
        ctx.push(*rows)
        if rows_keep is None:
            rows_keep = rows
    t_fill = time.perf_counter() - t_fill

    upl = max(1, min(args.updates_per_launch, 256))

    def run_updates(n):
        # the trainer's `for _ in range(updates_per_step)` loop: `upl` updates per launch
        full, rem = divmod(n, upl)
        for _ in range(full):
            ctx.step_many_async(args.batch, upl)
        if rem:
            ctx.step_many_async(args.batch, rem)

    # every graph the timed loop replays is captured, instantiated and replayed once
    # before the first timed window, whatever --warmup is
    for n in graph_sizes(args.steps, upl):
        ctx.step_many_async(args.batch, n)
    run_updates(args.warmup)
    ctx.synchronize()
    torch.cuda.synchronize()

    def window():
        t0 = time.perf_counter()
        run_updates(args.steps)
        losses = ctx.fetch_losses(args.steps)      # D2H of every loss, inside the timed region
        ctx.synchronize()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        assert losses.shape == (args.steps, 3) and np.all(np.isfinite(losses)), losses[-3:]
        return dt

    dt, dts = median_windows(window, args.windows)
    graphs = ctx.get_scalar(L.S_GRAPH_COUNT)
    if args.profile_only:
        emit(json.dumps({"steps": args.steps, "windows": args.windows,
                         "ms_per_step": 1e3 * dt / args.steps}))
        return
    sps = args.steps / dt

    # one update per launch (update_parameters_async), and the API-faithful mode with
    # the losses synced every update (sac_imp.py:140-144 .item())
    n_one = max(200, args.steps // 2)      # (~30 ms: host scheduling noise averages out)
    ctx.step_async(args.batch)
    ctx.synchronize()
    t1 = time.perf_counter()
    for _ in range(n_one):
        ctx.step_async(args.batch)
    ctx.fetch_losses(n_one)
    ctx.synchronize()
    one_sps = n_one / (time.perf_counter() - t1)
    n_sync = max(200, args.steps // 4)
    t1 = time.perf_counter()
    for _ in range(n_sync):
        ctx.step(args.batch)
    sync_sps = n_sync / (time.perf_counter() - t1)

    roof = None
    peak = PEAK_BF16_MFMA_TFLOPS if wl["dtype"] == "bf16" else PEAK_FP32_MFMA_TFLOPS
    if not args.no_roofline:
        # the timed graph's GPU time per update, for the instrumentation correction: 10
        # launches back to back, one wait (the window above also pays fetch + sync each)
        ctx.synchronize()
        reps = []
        for _ in range(3):
            t1 = time.perf_counter()
            for _ in range(10):
                ctx.step_many_async(args.batch, upl)
            ctx.synchronize()
            reps.append((time.perf_counter() - t1) / (10 * upl))
        roof = roofline_object(ctx, args, wl, peak, step_us_real=1e6 * float(np.median(reps)))
    flops = necessary_flops(S, A, H, args.batch, wl["n_hidden"])
    loop = None if args.no_trainer_loop else trainer_loop(wl)
    loop_f = None if args.no_trainer_loop else trainer_loop(wl, sync_python_random=True)
    cpu = None
    if not args.no_cpu_baseline:
        n_cpu = min(fill, 1_000_000)
        cpu_rows = tuple(x[:n_cpu] for x in synth(n_cpu, 7, S, A))
        cpu = cpu_baseline(cpu_rows, seconds=args.cpu_seconds, batch=args.batch, per=per,
                           n_hidden=wl["n_hidden"])
    env = "Humanoid-v5" if args.config != 5 else "NAO-walk"
    out = {
        "metric": f"SAC gradient-steps/sec, {env} batch={args.batch} (obs {S}, act {A}, hidden {H})",
        "value": round(sps, 2), "unit": "grad-steps/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "windows": args.windows,
        "window_ms_min_med_max": [round(1e3 * min(dts), 3), round(1e3 * dt, 3), round(1e3 * max(dts), 3)],
        "ms_per_step": round(1e3 / sps, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": wl["dtype"], "data": "synthetic",
        "config": {"workload": wl["workload"] + (" [networks_model2: 3 hidden layers]"
                                                 if wl["n_hidden"] == 3 else ""),
                   "state_dim": S, "action_dim": A, "hidden": H, "n_hidden": wl["n_hidden"],
                   "global_batch": args.batch, "replay_fill": fill, "parallelism": "single GPU"},
        "updates_per_launch": upl,
        "graphs_cached": int(graphs),
        "one_update_per_launch_steps_per_s": round(one_sps, 2),
        "api_faithful_steps_per_s": round(sync_sps, 2),
        "mfma_util_step": round(flops * sps / 1e12 / peak, 4),
        "necessary_gflop_per_step": round(flops / 1e9, 4),
        "trainer_loop": loop,
        "trainer_loop_faithful": loop_f,
        "roofline": roof, "cpu_baseline": cpu,
        "fill_seconds": round(t_fill, 2),
    }
    emit(json.dumps(out))


if __name__ == "__main__":
    main()
