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

    def phase(self, p: int, batch: int, grad_scale: float, parity: int = 0,
              have_batch: bool = False, ride_next: bool = False) -> None:
        self.ctx.step_phase(batch, p, grad_scale, parity, have_batch, ride_next)

    def ride_possible(self, batch: int) -> bool:
        return self.ctx.ride_possible(batch)


class DataParallelUpdate:
    """Callable running one update across the process group (its actor Adam is
    deferred into the next call; ``flush()`` completes it)."""

    def __init__(self, backend, group=None):
        self.backend = backend
        self.group = group
        self.world = dist.get_world_size(group)
        self._pending = None       # batch of an update whose phase 2 has not run
        # ride-along sequence (begin_sequence): the next update's sampling + gather run
        # inside this update's phase-1 launches, into the other minibatch buffer set
        self._seq_left = 0
        self._parity = 0
        self._have = False

    def begin_sequence(self, n: int, batch: int) -> None:
        """The next `n` calls form one uninterrupted sequence (nothing touches the replay
        buffer or the sampling stream in between, e.g. one captured graph): updates
        1..n-1 get their minibatch from the previous update's ride-along work."""
        ok = getattr(self.backend, "ride_possible", None)
        self._seq_left = n if (ok is not None and ok(batch)) else 0
        self._parity, self._have = 0, False

    def __call__(self, batch: int) -> None:
        b, scale = self.backend, 1.0 / self.world
        ride_next = self._seq_left > 1
        kw = {}
        if self._seq_left > 0:
            kw = dict(parity=self._parity, have_batch=self._have)
        if self._pending is not None and getattr(b, "supports_fused_tail", False):
            b.phase(3, batch, scale, **kw)
        else:
            self.flush()
            b.phase(0, batch, scale, **kw)
        self._pending = None
        dist.all_reduce(b.critic_grads, op=dist.ReduceOp.SUM, group=self.group)
        if self._seq_left > 0:
            b.phase(1, batch, scale, parity=self._parity, ride_next=ride_next)
            self._seq_left -= 1
            self._have = ride_next
            self._parity = self._parity ^ 1 if ride_next else 0
        else:
            b.phase(1, batch, scale)
        dist.all_reduce(b.actor_grads, op=dist.ReduceOp.SUM, group=self.group)
        self._pending = batch

    def flush(self) -> None:
        if self._pending is not None:
            self.backend.phase(2, self._pending, 1.0 / self.world)
            self._pending = None


class CapturedDataParallelUpdates:
    """Runs data-parallel updates as replays of torch.cuda.CUDAGraphs, each holding `n`
    consecutive updates — library launches and RCCL all-reduces — on one dedicated
    stream (the trainer's updates_per_step loop without per-update host launches).
    Every rank captures the same sequence, so the collectives pair up across ranks on
    replay.  Results are bit-identical to the eager driver (tests/test_gpu_parity.py)."""

    def __init__(self, ctx, device: torch.device, batch: int, group=None):
        self.device, self.batch = device, batch
        self.stream = torch.cuda.Stream(device)
        with torch.cuda.stream(self.stream):
            self.backend = GpuBackend(ctx, device)
        ctx.set_stream(self.stream.cuda_stream)
        self.upd = DataParallelUpdate(self.backend, group)
        self.graphs = {}
        # one eager update on the capture stream first: the library's phase graphs and
        # the communicator's buffers exist before any capture begins
        with torch.cuda.stream(self.stream):
            self.upd(batch)
            self.upd.flush()
        torch.cuda.synchronize(device)

    def _graph(self, n: int):
        g = self.graphs.get(n)
        if g is None:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=self.stream):
                self.upd.begin_sequence(n, self.batch)
                for _ in range(n):
                    self.upd(self.batch)
                self.upd.flush()
            self.graphs[n] = g
        return g

    def prepare(self, *sizes: int) -> None:
        for n in sizes:
            if n > 0:
                self._graph(n)

    def run(self, updates: int, per_launch: int) -> None:
        full, rem = divmod(updates, per_launch)
        for _ in range(full):
            self._graph(per_launch).replay()
        if rem:
            self._graph(rem).replay()


def run_dp_bench(args, rank: int, world: int, local_rank: int, emit=print):
    """bench.py --gpus N under torch.distributed.run (one rank per GPU)."""
    import bench as B
    from sacmi import Config, Context

    torch.cuda.set_device(local_rank)
    device = torch.device("cuda", local_rank)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=device)
    wl = B.workload(args)
    S, A, H = wl["S"], wl["A"], wl["H"]
    fill = args.fill // world                       # this rank's replay shard
    ctx = Context(Config(S, A, H, max_batch=args.batch, capacity=fill, seed=1000 + rank,
                         n_hidden=wl["n_hidden"], compute_dtype=wl["dtype"]), local_rank)
    B.init_agent(ctx, 0)                            # identical replicas
    key = np.random.default_rng(77 + rank).integers(0, 2**32, size=624, dtype=np.uint32)
    ctx.set_mt(0, key, 624)                         # per-shard sampling stream
    chunk = 100_000
    for c0 in range(0, fill, chunk):
        ctx.push(*B.synth(min(chunk, fill - c0), 5000 + rank * 7919 + c0, S, A))
    per_launch = max(1, min(args.updates_per_launch, 256))
    captured = None
    native = getattr(args, "dp_native", False)
    if native:
        # the library issues the all-reduces itself (sacmi_step_dp): RCCL unique id from
        # rank 0, broadcast over the process group
        uid = torch.zeros(128, dtype=torch.uint8, device=device)
        if rank == 0:
            uid.copy_(torch.frombuffer(bytearray(Context.allreduce_unique_id()), dtype=torch.uint8))
        dist.broadcast(uid, 0)
        ctx.allreduce_init(bytes(uid.cpu().numpy().tobytes()), rank, world)
        for n in {min(per_launch, args.steps), args.steps % per_launch, args.warmup % per_launch}:
            if n > 0:
                ctx.step_dp(args.batch, n)        # build the graphs (the updates are warm-up)
        ctx.synchronize()

        def run(k):
            full, rem = divmod(k, per_launch)
            for _ in range(full):
                ctx.step_dp(args.batch, per_launch)
            if rem:
                ctx.step_dp(args.batch, rem)
    elif os.environ.get("SACMI_DP_GRAPH", "1") == "1":
        try:
            captured = CapturedDataParallelUpdates(ctx, device, args.batch)
            captured.prepare(min(per_launch, args.steps), args.steps % per_launch,
                             args.warmup % per_launch)
        except Exception as e:                     # capture unsupported: eager driver
            if rank == 0:
                print(f"sacmi.dp: graph capture failed ({e}); eager updates", flush=True)
            captured = None
            torch.cuda.synchronize()
    if native:
        pass
    elif captured is None:
        upd = DataParallelUpdate(GpuBackend(ctx, device))

        def run(k):
            for _ in range(k):
                upd(args.batch)
            upd.flush()
    elif captured is not None:
        def run(k):
            captured.run(k, per_launch)
    run(args.warmup)
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    dt = torch.tensor([time.perf_counter() - t0], device=device)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    dt = float(dt.item())
    # replicas must have stayed identical: compare a parameter checksum across ranks
    w = torch.from_numpy(ctx.get_net("policy")["fc2.weight"]).to(device).double()
    chk = torch.stack([w.sum(), (w * w).sum()])
    allchk = [torch.zeros_like(chk) for _ in range(world)]
    dist.all_gather(allchk, chk)
    replicas_equal = all(bool(torch.equal(allchk[0], c)) for c in allchk)
    if rank == 0:
        iters = args.steps / dt
        value = world * iters
        flops = B.necessary_flops(S, A, H, args.batch, wl["n_hidden"])
        peak = B.PEAK_BF16_MFMA_TFLOPS if wl["dtype"] == "bf16" else B.PEAK_FP32_MFMA_TFLOPS
        env = "Humanoid-v5" if args.config != 5 else "NAO-walk"
        out = {
            "metric": f"SAC gradient-steps/sec, {env} batch={args.batch} (obs {S}, act {A}, hidden {H})",
            "value": round(value, 2), "unit": f"grad-steps/s (batch-{args.batch} per GPU)",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1e3 * dt / args.steps, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": wl["dtype"], "data": "synthetic",
            "config": {"workload": wl["workload"] + f"; {world} ranks: per-GPU replay shard + "
                                   "RCCL gradient all-reduce over xGMI (uniform replay per shard)",
                       "state_dim": S, "action_dim": A, "hidden": H, "n_hidden": wl["n_hidden"],
                       "global_batch": args.batch * world, "replay_fill": fill * world,
                       "parallelism": f"dp{world}"},
            "iterations_per_s": round(iters, 2),
            "updates_per_launch": per_launch if (captured or native) else 1,
            "dp_graph": captured is not None or native,
            "dp_driver": "library (sacmi_step_dp: RCCL issued by libsacmi)" if native
                         else "torch.distributed (RCCL) around sacmi phases",
            "mfma_util_step": round(flops * value / 1e12 / peak / world, 4),
            "replicas_bitwise_equal": replicas_equal,
            "roofline": None, "cpu_baseline": None,
        }
        emit(json.dumps(out))
    dist.barrier()
    dist.destroy_process_group()
