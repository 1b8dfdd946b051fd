"""Object wrapper over one libsacmi context (one agent on one GPU)."""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass

import numpy as np

from . import _lib as L

NET_IDS = {"policy": L.POLICY, "q1": L.Q1, "q2": L.Q2, "q1_target": L.Q1_TARGET,
           "q2_target": L.Q2_TARGET}
SLOTS = {"param": L.SLOT_PARAM, "grad": L.SLOT_GRAD, "m": L.SLOT_ADAM_M, "v": L.SLOT_ADAM_V}
COMPUTE_DTYPES = {"fp32": L.COMPUTE_FP32, "bf16": L.COMPUTE_BF16}


def layer_names(net: str, n_hidden: int = 2):
    """state_dict layer names in layer-index order: networks_model1.py:14-17,46-50
    (n_hidden=2), networks_model2.py:23-27,57-62 (n_hidden=3)."""
    hid = [f"fc{i}" for i in range(1, n_hidden + 1)]
    return hid + (["mean", "log_std"] if net == "policy" else [f"fc{n_hidden + 1}"])


def net_keys(net: str, n_hidden: int = 2):
    for layer, name in enumerate(layer_names(net, n_hidden)):
        yield f"{name}.weight", layer, 0
        yield f"{name}.bias", layer, 1


@dataclass
class Config:
    state_dim: int
    action_dim: int
    hidden_dim: int = 256
    max_batch: int = 4096
    gamma: float = 0.99
    tau: float = 0.005
    lr: float = 3e-4
    alpha: float = 0.2
    automatic_entropy_tuning: bool = True
    replay: str = "uniform"
    action_low: float = -0.4
    action_high: float = 0.4
    capacity: int = 1_000_000
    per_alpha: float = 0.6
    per_beta_start: float = 0.4
    per_beta_frames: float = 100000
    seed: int = 0
    n_hidden: int = 2              # 2: networks_model1, 3: networks_model2
    compute_dtype: str = "fp32"    # "fp32" | "bf16" (MLP GEMM operands; fp32 accumulate)

    def to_c(self) -> L.SacmiConfig:
        c = L.SacmiConfig()
        c.state_dim, c.action_dim, c.hidden_dim = self.state_dim, self.action_dim, self.hidden_dim
        c.max_batch = self.max_batch
        c.gamma, c.tau, c.lr, c.alpha = self.gamma, self.tau, self.lr, self.alpha
        c.auto_entropy = int(bool(self.automatic_entropy_tuning))
        c.replay_kind = L.REPLAY_PER if self.replay == "per" else L.REPLAY_UNIFORM
        c.action_low, c.action_high = self.action_low, self.action_high
        c.capacity = int(self.capacity)
        c.per_alpha, c.per_beta_start = self.per_alpha, self.per_beta_start
        c.per_beta_frames = float(self.per_beta_frames)
        c.seed = int(self.seed) & ((1 << 64) - 1)
        c.n_hidden = int(self.n_hidden)
        if self.compute_dtype not in COMPUTE_DTYPES:
            raise ValueError(f"compute_dtype must be one of {sorted(COMPUTE_DTYPES)}")
        c.compute_dtype = COMPUTE_DTYPES[self.compute_dtype]
        return c


def setsize(k: int) -> int:
    """random.py:488-490 (the pool/set branch threshold of random.sample)."""
    s = 21
    if k > 5:
        s += 4 ** math.ceil(math.log(k * 3, 4))
    return s


class Context:
    """Owns a ``sacmi_ctx``; every method is one C-ABI call."""

    def __init__(self, cfg: Config, device: int = 0):
        self.cfg = cfg
        self.device = device
        self._lib = L.load()
        h = ctypes.c_void_p()
        ccfg = cfg.to_c()
        L.call("sacmi_create", ctypes.byref(ccfg), int(device), ctypes.byref(h))
        self._h = h

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            L.call("sacmi_destroy", self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- streams -----------------------------------------------------------------
    def set_stream(self, stream_handle: int | None):
        L.call("sacmi_set_stream", self._h, ctypes.c_void_p(stream_handle or 0))

    def synchronize(self):
        L.call("sacmi_synchronize", self._h)

    # -- tensors -----------------------------------------------------------------
    def numel(self, net: str, layer: int, part: int) -> int:
        n = ctypes.c_int64()
        L.call("sacmi_tensor_numel", self._h, NET_IDS[net], layer, part, ctypes.byref(n))
        return n.value

    def get_tensor(self, slot: str, net: str, layer: int, part: int, shape) -> np.ndarray:
        out = np.empty(shape, np.float32)
        L.call("sacmi_get_tensor", self._h, SLOTS[slot], NET_IDS[net], layer, part, L.fptr(out),
               out.size)
        return out

    def set_tensor(self, slot: str, net: str, layer: int, part: int, value) -> None:
        v = np.ascontiguousarray(value, dtype=np.float32)
        L.call("sacmi_set_tensor", self._h, SLOTS[slot], NET_IDS[net], layer, part, L.fptr(v),
               v.size)

    def get_net(self, net: str, slot: str = "param", shapes: dict | None = None) -> dict:
        out = {}
        for key, layer, part in net_keys(net, self.cfg.n_hidden):
            n = self.numel(net, layer, part)
            shp = shapes[key] if shapes else (n,)
            out[key] = self.get_tensor(slot, net, layer, part, shp)
        return out

    def set_net(self, net: str, sd: dict, slot: str = "param") -> None:
        for key, layer, part in net_keys(net, self.cfg.n_hidden):
            self.set_tensor(slot, net, layer, part, np.asarray(sd[key]))

    def get_scalar(self, which: int) -> float:
        v = ctypes.c_double()
        L.call("sacmi_get_scalar", self._h, which, ctypes.byref(v))
        return v.value

    def set_scalar(self, which: int, value: float) -> None:
        L.call("sacmi_set_scalar", self._h, which, float(value))

    def rng_seed_device(self, seed: int, offset: int = 0) -> None:
        """Re-key the perf-mode policy noise (Philox seed, per-update counter start)."""
        L.call("sacmi_rng_seed_device", self._h, int(seed), int(offset))

    # -- replay --------------------------------------------------------------------
    def push(self, s, a, r, s2, d) -> None:
        S, A = self.cfg.state_dim, self.cfg.action_dim
        s = np.ascontiguousarray(s, np.float32).reshape(-1, S)
        n = s.shape[0]
        a = np.ascontiguousarray(a, np.float32).reshape(n, A)
        r = np.ascontiguousarray(r, np.float32).reshape(n)
        s2 = np.ascontiguousarray(s2, np.float32).reshape(n, S)
        d = np.ascontiguousarray(np.asarray(d).astype(bool), np.uint8).reshape(n)
        L.call("sacmi_push", self._h, L.fptr(s), L.fptr(a), L.fptr(r), L.fptr(s2), L.u8ptr(d), n)

    def push_packed(self, rows: np.ndarray, n: int) -> None:
        """n packed rows (float32 [>= n][2S + A + 2]: s | a | r | s2 | d), copy-in."""
        S, A = self.cfg.state_dim, self.cfg.action_dim
        assert rows.dtype == np.float32 and rows.flags.c_contiguous and rows.shape[-1] == 2 * S + A + 2
        assert rows.size >= n * (2 * S + A + 2)
        L.call("sacmi_push_packed", self._h, rows.ctypes.data, int(n))

    def __len__(self) -> int:
        n = ctypes.c_int64()
        L.call("sacmi_len", self._h, ctypes.byref(n))
        return n.value

    def replay_clear(self) -> None:
        """Empty the ring (the checkpoint restore's buffer replacement, sac_imp.py:229-230)."""
        L.call("sacmi_replay_clear", self._h)

    def get_rows(self, idx):
        idx = np.ascontiguousarray(idx, np.int64)
        n = idx.size
        S, A = self.cfg.state_dim, self.cfg.action_dim
        s = np.empty((n, S), np.float32); s2 = np.empty((n, S), np.float32)
        a = np.empty((n, A), np.float32); r = np.empty(n, np.float32); d = np.empty(n, np.uint8)
        L.call("sacmi_get_rows", self._h, L.i64ptr(idx), n, L.fptr(s), L.fptr(a), L.fptr(r),
               L.fptr(s2), L.u8ptr(d))
        return s, a, r, s2, d.astype(bool)

    def get_slots(self, slots):
        """Rows at ring slots (PER indices)."""
        idx = np.ascontiguousarray(slots, np.int64)
        n = idx.size
        S, A = self.cfg.state_dim, self.cfg.action_dim
        s = np.empty((n, S), np.float32); s2 = np.empty((n, S), np.float32)
        a = np.empty((n, A), np.float32); r = np.empty(n, np.float32); d = np.empty(n, np.uint8)
        L.call("sacmi_get_slots", self._h, L.i64ptr(idx), n, L.fptr(s), L.fptr(a), L.fptr(r),
               L.fptr(s2), L.u8ptr(d))
        return s, a, r, s2, d.astype(bool)

    # -- rng -----------------------------------------------------------------------
    def set_mt(self, stream: int, key, pos: int) -> None:
        k = np.ascontiguousarray(key, np.uint32)
        assert k.shape == (624,)
        L.call("sacmi_rng_set_mt", self._h, stream, L.u32ptr(k), int(pos))

    def get_mt(self, stream: int):
        k = np.empty(624, np.uint32)
        p = ctypes.c_int32()
        L.call("sacmi_rng_get_mt", self._h, stream, L.u32ptr(k), ctypes.byref(p))
        return k, p.value

    def sample_indices(self, batch: int) -> np.ndarray:
        out = np.empty(batch, np.int64)
        L.call("sacmi_sample_indices", self._h, int(batch), L.i64ptr(out))
        return out

    # -- the update ------------------------------------------------------------------
    def step(self, batch: int, idx=None, eps1=None, eps2=None, want_losses: bool = True):
        A = self.cfg.action_dim
        idx_a = None if idx is None else np.ascontiguousarray(idx, np.int64)
        e1 = None if eps1 is None else np.ascontiguousarray(eps1, np.float32).reshape(batch, A)
        e2 = None if eps2 is None else np.ascontiguousarray(eps2, np.float32).reshape(batch, A)
        out = np.zeros(3, np.float32) if want_losses else None
        L.call("sacmi_step", self._h, int(batch), L.i64ptr(idx_a), L.fptr(e1), L.fptr(e2),
               L.fptr(out))
        return out

    def step_launch(self, batch: int) -> None:
        """First half of step(batch) (device indices + noise): enqueue and return."""
        L.call("sacmi_step_launch", self._h, int(batch))

    def step_wait(self) -> np.ndarray:
        """Second half: wait for the launched update; its losses (ValueError on ENAN)."""
        out = np.zeros(3, np.float32)
        L.call("sacmi_step_wait", self._h, L.fptr(out))
        return out

    def step_async(self, batch: int) -> None:
        L.call("sacmi_step_async", self._h, int(batch))

    def step_many_async(self, batch: int, n_updates: int) -> None:
        """n_updates consecutive updates in one launch (trainer.py:203-204 loop)."""
        L.call("sacmi_step_many_async", self._h, int(batch), int(n_updates))

    def fetch_losses(self, max_steps: int) -> np.ndarray:
        out = np.zeros((max_steps, 3), np.float32)
        n = ctypes.c_int32()
        L.call("sacmi_fetch_losses", self._h, L.fptr(out), int(max_steps), ctypes.byref(n))
        return out[:n.value]

    def step_phase(self, batch: int, phase: int, grad_scale: float = 1.0, parity: int = 0,
                   have_batch: bool = False, ride_next: bool = False) -> None:
        if parity or have_batch or ride_next:
            L.call("sacmi_step_phase_ex", self._h, int(batch), int(phase), float(grad_scale),
                   int(parity), int(bool(have_batch)), int(bool(ride_next)))
        else:
            L.call("sacmi_step_phase", self._h, int(batch), int(phase), float(grad_scale))

    # -- native data parallel (RCCL issued by the library) ----------------------------
    @staticmethod
    def allreduce_unique_id() -> bytes:
        """rank 0: a fresh RCCL unique id (SACMI_RCCL_ID_BYTES bytes) to hand to every rank."""
        buf = ctypes.create_string_buffer(L.RCCL_ID_BYTES)
        L.call("sacmi_allreduce_unique_id", buf, L.RCCL_ID_BYTES)
        return buf.raw

    def allreduce_init(self, unique_id: bytes, rank: int, world: int) -> None:
        L.call("sacmi_allreduce_init", self._h, unique_id, len(unique_id), int(rank), int(world))

    def dp_loopback_init(self, world: int) -> None:
        """Test hook: step_dp on this one context with every all-reduce replaced by an
        in-place x world (identical shards on `world` ranks), see include/sacmi.h."""
        L.call("sacmi_dp_loopback_init", self._h, int(world))

    def step_dp(self, batch: int, n_updates: int = 1) -> None:
        """n complete data-parallel updates (phases + library-issued RCCL collectives)."""
        L.call("sacmi_step_dp", self._h, int(batch), int(n_updates))

    def dp_set_sharded(self, on: bool) -> None:
        """Sharded optimizer step (reduce-scatter -> Adam on 1/world -> all-gather) or the
        all-reduce form of step_dp (include/sacmi.h)."""
        L.call("sacmi_dp_set_sharded", self._h, 1 if on else 0)

    def dp_sharded(self) -> bool:
        out = ctypes.c_int32()
        L.call("sacmi_dp_sharded", self._h, ctypes.byref(out))
        return bool(out.value)

    def dp_sync_state(self) -> None:
        """Collective: gather the sharded Adam moments on every rank (before reading them)."""
        L.call("sacmi_dp_sync_state", self._h)

    def ride_possible(self, batch: int) -> bool:
        out = ctypes.c_int32()
        L.call("sacmi_step_ride_possible", self._h, int(batch), ctypes.byref(out))
        return bool(out.value)

    def read_activation(self, pass_: int, layer: int, batch: int) -> np.ndarray:
        """The last update's hidden activations (sacmi.h sacmi_read_activation): passes 0-2
        -> [2, batch, hidden] (q1, q2), pass 3 (policy on [s'; s]) -> [2 * batch, hidden]."""
        H = self.cfg.hidden_dim
        out = np.zeros(2 * batch * H, np.float32)
        L.call("sacmi_read_activation", self._h, int(pass_), int(layer), int(batch), L.fptr(out), out.size)
        return out.reshape((2 * batch, H) if pass_ == 3 else (2, batch, H))

    def read_batch(self, batch: int):
        """(idx[batch] int64, eps[2 * batch, A] float32) of the last device-sampled update of
        `batch` rows in batch set 0 (sacmi.h sacmi_read_batch): eps rows [0, batch) noise of
        policy.sample(next_state), rows [batch, 2 batch) of policy.sample(state)."""
        A = self.cfg.action_dim
        idx = np.zeros(batch, np.int64)
        eps = np.zeros(2 * batch * A, np.float32)
        L.call("sacmi_read_batch", self._h, int(batch),
               idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), L.fptr(eps), eps.size)
        return idx, eps.reshape(2 * batch, A)

    def act16(self, batch: int) -> bool:
        """Whether updates of this batch keep their activations in bf16 (sacmi.h)."""
        out = ctypes.c_int32()
        L.call("sacmi_step_act16", self._h, int(batch), ctypes.byref(out))
        return bool(out.value)

    def grad_arena_numel(self) -> int:
        n = ctypes.c_int64()
        L.call("sacmi_grad_arena_numel", self._h, ctypes.byref(n))
        return n.value

    def attach_grad_arena(self, device_ptr: int, numel: int) -> None:
        L.call("sacmi_attach_grad_arena", self._h, ctypes.c_void_p(device_ptr), int(numel))

    def grad_buffer(self, which: int):
        p = ctypes.c_void_p()
        n = ctypes.c_int64()
        L.call("sacmi_grad_buffer", self._h, which, ctypes.byref(p), ctypes.byref(n))
        return p.value, n.value

    # -- PER -------------------------------------------------------------------------
    def per_sample(self, batch: int, u=None):
        n = min(batch, len(self))
        idx = np.empty(n, np.int64)
        w = np.empty(n, np.float32)
        u_a = None if u is None else np.ascontiguousarray(u, np.float64)
        L.call("sacmi_per_sample", self._h, int(batch), L.dptr(u_a), L.i64ptr(idx), L.fptr(w))
        return idx, w

    def per_update(self, idx, values) -> None:
        """priorities[idx[i]] = values[i], last duplicate wins (values already hold the
        reference's float32(float(p) + 1e-6))."""
        idx = np.ascontiguousarray(idx, np.int64)
        p = np.ascontiguousarray(values, np.float32).reshape(-1)
        L.call("sacmi_per_update", self._h, L.i64ptr(idx), L.fptr(p), idx.size)

    def per_priorities(self, n: int | None = None) -> np.ndarray:
        n = self.cfg.capacity if n is None else n
        out = np.empty(n, np.float32)
        L.call("sacmi_per_get_priorities", self._h, L.fptr(out), n)
        return out

    def per_set_priorities(self, prio) -> None:
        p = np.ascontiguousarray(prio, np.float32)
        L.call("sacmi_per_set_priorities", self._h, L.fptr(p), p.size)

    # -- diagnostics -------------------------------------------------------------------
    def profile_step(self, batch: int, iters: int = 10):
        """[(site, mean_ms, flops_per_launch)] over `iters` eager updates (HIP events)."""
        mx = 64
        names = ctypes.create_string_buffer(32 * mx)
        ms = np.zeros(mx, np.float32)
        fl = np.zeros(mx, np.float64)
        n = ctypes.c_int32()
        L.call("sacmi_profile_step", self._h, int(batch), int(iters), names, L.fptr(ms),
               L.dptr(fl), mx, ctypes.byref(n))
        raw = names.raw
        return [(raw[32 * i:32 * i + 32].split(b"\0")[0].decode(), float(ms[i]), float(fl[i]))
                for i in range(n.value)]

    def profile_sites(self, batch: int, reps: int = 50):
        """[(site, mean_us, flops_per_launch, bytes_per_launch)]: each launch site alone,
        `reps` times in one hipGraph, timed with HIP events on the context stream
        (advances the state)."""
        mx = 64
        names = ctypes.create_string_buffer(32 * mx)
        us = np.zeros(mx, np.float32)
        fl = np.zeros(mx, np.float64)
        by = np.zeros(mx, np.float64)
        n = ctypes.c_int32()
        L.call("sacmi_profile_sites", self._h, int(batch), int(reps), names, L.fptr(us),
               L.dptr(fl), L.dptr(by), mx, ctypes.byref(n))
        raw = names.raw
        return [(raw[32 * i:32 * i + 32].split(b"\0")[0].decode(), float(us[i]), float(fl[i]),
                 float(by[i])) for i in range(n.value)]

    def profile_timeline(self, batch: int, n_updates: int, data_parallel: bool = False):
        """Launch timeline of `n_updates` updates as step_many_async runs them (one graph,
        every kernel stamping its first-workgroup entry / last-workgroup exit on the GPU's
        100 MHz clock).  Returns (kernels, graph_us): kernels = [dict(site, site_idx,
        kernel, grid, start_us, end_us, flops, bytes)] in launch order (the site's algorithmic
        FLOPs / bytes on its first kernel); graph_us = HIP-event time of the
        replay.  Advances the state by 2 * n_updates updates.  ``data_parallel``: the
        sequence step_dp replays (phases + RCCL all-reduces; every rank must call)."""
        fn = "sacmi_profile_timeline_dp" if data_parallel else "sacmi_profile_timeline"
        mx = 64 * n_updates * 8
        names = ctypes.create_string_buffer(32 * mx)
        kind = np.zeros(mx, np.int32); grid = np.zeros(mx, np.int32); site = np.zeros(mx, np.int32)
        t0 = np.zeros(mx, np.float64); t1 = np.zeros(mx, np.float64)
        fl = np.zeros(mx, np.float64); by = np.zeros(mx, np.float64)
        n = ctypes.c_int32()
        g = ctypes.c_double()
        L.call(fn, self._h, int(batch), int(n_updates), mx, names,
               L.i32ptr(kind), L.i32ptr(grid), L.i32ptr(site), L.dptr(t0), L.dptr(t1), L.dptr(fl),
               L.dptr(by), ctypes.byref(n), ctypes.byref(g))
        raw = names.raw
        out = [dict(site=raw[32 * i:32 * i + 32].split(b"\0")[0].decode(), site_idx=int(site[i]),
                    kernel=L.TL_KINDS.get(int(kind[i]), str(int(kind[i]))), grid=int(grid[i]),
                    start_us=float(t0[i]), end_us=float(t1[i]), flops=float(fl[i]),
                    bytes=float(by[i])) for i in range(n.value)]
        return out, g.value

    # -- act -------------------------------------------------------------------------
    def act(self, states, deterministic: bool, eps=None) -> np.ndarray:
        S, A = self.cfg.state_dim, self.cfg.action_dim
        s = np.ascontiguousarray(states, np.float32).reshape(-1, S)
        n = s.shape[0]
        if n == 1 and eps is None:     # the env-rate call: reused buffers and pointers
            if getattr(self, "_act1", None) is None:
                bufs = (np.empty(S, np.float32), np.empty((1, A), np.float32))
                self._act1 = bufs + (L.fptr(bufs[0]), L.fptr(bufs[1]))
            bi, bo, pi, po = self._act1
            bi[...] = s[0]
            L.call("sacmi_act", self._h, pi, 1, int(bool(deterministic)), None, po)
            return bo.copy()
        e = None if eps is None else np.ascontiguousarray(eps, np.float32).reshape(n, A)
        out = np.empty((n, A), np.float32)
        L.call("sacmi_act", self._h, L.fptr(s), n, int(bool(deterministic)), L.fptr(e), L.fptr(out))
        return out
