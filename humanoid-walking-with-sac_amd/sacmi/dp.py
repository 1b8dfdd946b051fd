"""Data-parallel SAC updates: one process per GPU, RCCL gradient all-reduce.

SURVEY §8(e): every loss of ``update_parameters`` is a batch mean, so with equal
per-rank batches the mean of the per-rank gradients equals the gradient of the
concatenated global batch.  Each rank samples from its own HBM replay shard; the
update is split where the reference has an ordering constraint (the actor must see
the post-Adam critics, sac_imp.py:101-125):

  phase 0  sample, gather, forward, critic backward   -> critic gradient buffer
           all_reduce(SUM) critic grads                 (RCCL over xGMI)
  phase 1  critic Adam (x 1/world) + Polyak, actor forward/backward -> actor buffer
           all_reduce(SUM) [policy grads | dL/dlog_alpha]
  phase 2  actor Adam (x 1/world) + alpha

Phase 2 of one update and phase 0 of the next have no collective between them, so the
driver defers phase 2 and launches it together with the next phase 0 (library phase 3);
``flush()`` runs a deferred phase 2 (before reading parameters).

Every rank applies the identical reduced gradient with the identical deterministic
kernels, so replicas stay bitwise identical.  The collectives run on tensors that
alias the library's gradient arena (torch allocates it, libsacmi adopts it), ordered
on torch's current stream, on which the library also runs.
"""
from __future__ import annotations

import json
import os
import time

import numpy as np
import torch
import torch.distributed as dist


class GpuBackend:
    """libsacmi context whose gradient arena is a torch tensor on ``device``."""

    def __init__(self, ctx, device: torch.device):
        self.ctx = ctx
        n = ctx.grad_arena_numel()
        self.arena = torch.zeros(n, dtype=torch.float32, device=device)
        ctx.attach_grad_arena(self.arena.data_ptr(), n)
        ctx.set_stream(torch.cuda.current_stream(device).cuda_stream)
        base = self.arena.data_ptr()
        views = []
        for which in (0, 1):
            ptr, numel = ctx.grad_buffer(which)
            off = (ptr - base) // 4
            views.append(self.arena.narrow(0, off, numel))
        self.critic_grads, self.actor_grads = views

    supports_fused_tail = True     # library phase 3 = phase 2 + next phase 0

    def phase(self, p: int, batch: int, grad_scale: float) -> None:
        self.ctx.step_phase(batch, p, grad_scale)


class DataParallelUpdate:
    """Callable running one update across the process group (its actor Adam is
    deferred into the next call; ``flush()`` completes it)."""

    def __init__(self, backend, group=None):
        self.backend = backend
        self.group = group
        self.world = dist.get_world_size(group)
        self._pending = None       # batch of an update whose phase 2 has not run

    def __call__(self, batch: int) -> None:
        b, scale = self.backend, 1.0 / self.world
        if self._pending is not None and getattr(b, "supports_fused_tail", False):
            b.phase(3, batch, scale)
        else:
            self.flush()
            b.phase(0, batch, scale)
        self._pending = None
        dist.all_reduce(b.critic_grads, op=dist.ReduceOp.SUM, group=self.group)
        b.phase(1, batch, scale)
        dist.all_reduce(b.actor_grads, op=dist.ReduceOp.SUM, group=self.group)
        self._pending = batch

    def flush(self) -> None:
        if self._pending is not None:
            self.backend.phase(2, self._pending, 1.0 / self.world)
            self._pending = None


def _native_comm(ctx, rank: int, device, group=None) -> None:
    """The library's own communicator over the same ranks (sacmi_allreduce_init): RCCL
    unique id from rank 0, broadcast over the process group."""
    from sacmi import Context
    uid = torch.zeros(128, dtype=torch.uint8, device=device)
    if rank == 0:
        uid.copy_(torch.frombuffer(bytearray(Context.allreduce_unique_id()), dtype=torch.uint8))
    dist.broadcast(uid, 0, group=group)
    ctx.allreduce_init(bytes(uid.cpu().numpy().tobytes()), rank, dist.get_world_size(group))


def run_dp_bench(args, rank: int, world: int, local_rank: int, emit=print):
    """bench.py --gpus N under torch.distributed.run (one rank per GPU): every rank owns a
    replay shard of fill/N rows (uniform, or prioritized for --config 3 / BASELINE configs[3]:
    each rank's PER sampler normalises over its own shard) and draws its own
    batch from it with its own MT streams; the critic and actor gradients are all-reduced
    over RCCL.  Timed as the median of windows of --steps updates (barrier + device sync on
    both sides, max over ranks)."""
    import bench as B
    from sacmi import Config, Context

    torch.cuda.set_device(local_rank)
    device = torch.device("cuda", local_rank)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=device)
    wl = B.workload(args)
    S, A, H = wl["S"], wl["A"], wl["H"]
    per = wl["replay"] == "per"
    fill = args.fill // world                       # this rank's replay shard
    ctx = Context(Config(S, A, H, max_batch=args.batch, capacity=fill, seed=1000 + rank,
                         replay=wl["replay"], n_hidden=wl["n_hidden"],
                         compute_dtype=wl["dtype"]), local_rank)
    B.init_agent(ctx, 0)                            # identical replicas
    for stream in (0, 1):                           # random.sample / numpy (PER) streams
        key = np.random.default_rng(77 + 31 * stream + rank).integers(0, 2**32, size=624,
                                                                      dtype=np.uint32)
        ctx.set_mt(stream, key, 624)                # per-shard sampling streams
    t_fill = time.perf_counter()
    chunk = 100_000
    for c0 in range(0, fill, chunk):
        ctx.push(*B.synth(min(chunk, fill - c0), 5000 + rank * 7919 + c0, S, A))
    t_fill = time.perf_counter() - t_fill
    per_launch = max(1, min(args.updates_per_launch, 256))
    sizes = B.graph_sizes(args.steps, per_launch)
    # default: the library's own RCCL sequence (sacmi_step_dp, one hipGraph per n updates).
    # --dp-torch: the torch.distributed driver, eager (torch's all-reduces between the
    # library's phase graphs).  Its torch.cuda.CUDAGraph-captured form was dropped: a world-1
    # run aborted in ProcessGroupNCCL's watchdog during a capture
    native = not getattr(args, "dp_torch", False)
    # the library's communicator: the native driver's collectives, and the roofline's
    # timeline of the data-parallel sequence (both paths)
    want_roof = not getattr(args, "no_roofline", False)
    sim = int(getattr(args, "dp_sim_world", 0) or 0)
    if sim:                                         # one GPU stands in for `sim` ranks
        # rank 0's work only, in BOTH optimizer forms (SACMI_DP_LOOPBACK_ONE_RANK, read at each
        # capture): the sharded form's Adam on rank 0's chunk, the collectives returning the
        # rank's own gradient with no stand-in kernels — without it the loopback steps all
        # `sim` chunks in turn, sim x a rank's optimizer work (round 5's dp_form_ab legs
        # differed by 42 % for that reason alone), and scales the gradients in place
        os.environ["SACMI_DP_LOOPBACK_ONE_RANK"] = "1"
        ctx.dp_loopback_init(sim)
    elif native or want_roof:
        _native_comm(ctx, rank, device)
    if native:
        for n in sizes:
            ctx.step_dp(args.batch, n)            # build the graphs (the updates are warm-up)
        ctx.synchronize()

        def run(k):
            full, rem = divmod(k, per_launch)
            for _ in range(full):
                ctx.step_dp(args.batch, per_launch)
            if rem:
                ctx.step_dp(args.batch, rem)
    else:
        upd = DataParallelUpdate(GpuBackend(ctx, device))

        def run(k):
            for _ in range(k):
                upd(args.batch)
            upd.flush()
    run(args.warmup)
    torch.cuda.synchronize()

    def window():
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(args.steps)
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()
        dt = torch.tensor([time.perf_counter() - t0], device=device)
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        return float(dt.item())

    dts = [window() for _ in range(args.windows)]
    dt = float(np.median(dts))

    def replicas_equal() -> bool:
        """replicas must have stayed identical: a parameter checksum across ranks"""
        w = torch.from_numpy(ctx.get_net("policy")["fc2.weight"]).to(device).double()
        chk = torch.stack([w.sum(), (w * w).sum()])
        allchk = [torch.zeros_like(chk) for _ in range(world)]
        dist.all_gather(allchk, chk)
        return all(bool(torch.equal(allchk[0], c)) for c in allchk)

    replicas_ok = replicas_equal()
    peak = B.PEAK_BF16_MFMA_TFLOPS if wl["dtype"] == "bf16" else B.PEAK_FP32_MFMA_TFLOPS
    roof = None
    if want_roof:
        # every rank replays the instrumented sequence (its graph holds the collectives)
        roof = B.roofline_object(ctx, args, wl, peak, data_parallel=True)
        torch.cuda.synchronize()
    # the other optimizer-step form on the same ranks, after the line's own measurement
    # (the line is the default form's): per-update time, the collectives' share of the
    # sequence (timeline gaps) and the replica check — the all-reduce vs the sharded
    # (ZeRO-1) form over real RCCL ranks (SACMI_BENCH_DP_FORM_AB=0: skipped)
    form_ab = None
    phases = world > 1 or sim or os.environ.get("SACMI_DP_PHASES_AT_WORLD1") is not None
    if native and phases and os.environ.get("SACMI_BENCH_DP_FORM_AB", "1") != "0":
        was = ctx.dp_sharded()
        form_ab = {"form": "sharded" if not was else "all-reduce"}
        # the switch and the first launch of each graph (its capture) are where one rank can
        # fail alone: every rank learns the outcome before any collective of the other form
        # runs, so all go on or all skip together (a rank that raised while the others wait
        # inside a collective would hang them)
        err = None
        try:
            ctx.dp_set_sharded(not was)
        except Exception as e:   # noqa: BLE001
            err = e
        bad = torch.tensor([0.0 if err is None else 1.0], device=device)
        dist.all_reduce(bad)
        if float(bad.item()) > 0:
            form_ab["error"] = (f"{type(err).__name__}: {err}" if err is not None
                                else "another rank could not switch")[:300]
            if err is None:
                ctx.dp_set_sharded(was)       # (leaving the sharded form: a collective — every
                                              #  rank that switched does this)
        else:
            # (a failure from here on, inside the other form's collectives, is re-raised: the
            # ranks cannot be kept in step past it; the original form is restored first)
            try:
                for n in sizes:
                    ctx.step_dp(args.batch, n)
                run(args.warmup)
                torch.cuda.synchronize()
                adts = [window() for _ in range(max(3, args.windows // 4))]
                adt = float(np.median(adts))
                form_ab.update({
                    "ms_per_step": round(1e3 * adt / args.steps, 4),
                    "value": round(world * args.steps / adt, 2),
                    "windows": len(adts),
                    "replicas_bitwise_equal": replicas_equal(),
                })
                if want_roof:
                    info = B.timeline_roofline(ctx, args.batch, per_launch, data_parallel=True)
                    form_ab["allreduce_us_per_step"] = round(info["allreduce_us"] / per_launch, 2)
                    form_ab["step_us_timeline"] = round(info["graph_us"] / per_launch, 2)
            finally:
                # (leaving the sharded form gathers the moments: a collective)
                ctx.dp_set_sharded(was)
                torch.cuda.synchronize()
    cpu = None
    # (the CPU baseline is timed on rank 0 at N = 1 only: the N > 1 lines carry none)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        n_cpu = min(fill * world, 1_000_000)
        cpu_rows = tuple(x[:n_cpu] for x in B.synth(n_cpu, 7, S, A))
        cpu = B.cpu_baseline(cpu_rows, seconds=args.cpu_seconds, batch=args.batch, per=per,
                             n_hidden=wl["n_hidden"])
        cpu["sample"] += "; one rank's batch (the per-GPU work of one data-parallel iteration)"
    if rank == 0:
        iters = args.steps / dt
        value = world * iters
        flops = B.necessary_flops(S, A, H, args.batch, wl["n_hidden"])
        env = "Humanoid-v5" if args.config != 5 else "NAO-walk"
        out = {
            "metric": f"SAC gradient-steps/sec, {env} batch={args.batch} (obs {S}, act {A}, hidden {H})",
            "value": round(value, 2), "unit": f"grad-steps/s (batch-{args.batch} per GPU)",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "windows": args.windows,
            "window_ms_min_med_max": [round(1e3 * min(dts), 3), round(1e3 * dt, 3),
                                      round(1e3 * max(dts), 3)],
            "ms_per_step": round(1e3 * dt / args.steps, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": wl["dtype"], "data": "synthetic",
            "config": {"workload": wl["workload"] + f"; {world} ranks: per-GPU replay shard of "
                                   f"{fill} rows ({'prioritized' if per else 'uniform'} replay "
                                   "per shard) + RCCL gradient all-reduce over xGMI",
                       "state_dim": S, "action_dim": A, "hidden": H, "n_hidden": wl["n_hidden"],
                       "global_batch": args.batch * world, "replay_fill": fill * world,
                       "replay": wl["replay"], "parallelism": f"dp{world}"},
            "iterations_per_s": round(iters, 2),
            "updates_per_launch": per_launch if native else 1,
            "dp_graph": native,
            "dp_driver": "library (sacmi_step_dp: RCCL issued by libsacmi)" if native
                         else "torch.distributed (RCCL) around sacmi phases",
            "dp_optimizer_step": ("sharded: reduce-scatter -> Adam on 1/world -> all-gather"
                                  if ctx.dp_sharded() else "all-reduce -> Adam on every rank"),
            "simulated_world": sim or None,
            "simulated_note": (f"one GPU runs rank 0's sequence of a {sim}-rank job, collectives "
                               "returning the rank's own gradient (no transfers, no stand-in "
                               "kernels; the sharded form's Adam on rank 0's chunk: "
                               "SACMI_DP_LOOPBACK_ONE_RANK): the per-rank work minus the "
                               "collectives" if sim else None),
            "mfma_util_step": round(flops * value / 1e12 / peak / world, 4),
            "replicas_bitwise_equal": replicas_ok,
            "dp_form_ab": form_ab,
            "roofline": roof, "cpu_baseline": cpu,
            "fill_seconds": round(t_fill, 2),
        }
        emit(json.dumps(out))
    dist.barrier()
    dist.destroy_process_group()
