"""Drop-in replay buffers (reference replay_buffer.py) backed by the HBM ring of a
libsacmi context.

* ``ReplayBuffer``: deque(maxlen=capacity) semantics (replay_buffer.py:5-22).
  ``sample`` is CPython's ``random.sample`` reproduced bit-exactly on the GPU
  (MT19937 stream + both sample branches); with ``sync_python_random=True`` the
  device stream is the interpreter's global ``random`` state (read before, written
  back after), so index sequences equal the reference's.
* ``PrioritizedReplayBuffer``: replay_buffer.py:25-90 (pow, normalise, inverse-CDF
  search, IS weights, priority updates), numpy's global RandomState as the uniform
  source when ``sync_numpy_random=True``.

Transitions are staged on the host by ``push`` (an env-rate call must not pay a PCIe
round trip) and flushed to HBM in one batched copy before any device use.  Values
are stored as float32 — exactly what the reference's update consumes after
``torch.FloatTensor`` (sac_imp.py:81-85).
"""
from __future__ import annotations

import random
from collections import deque

import numpy as np

from .core import Config, Context

_STAGE = 4096


class _Staged:
    def __init__(self, capacity: int, ctx: Context | None, replay: str):
        self.capacity = int(capacity)
        self._ctx = ctx
        self._replay = replay
        self._rows = []            # pending (s, a, r, s2, d)
        self._pack = None          # packed staging for sacmi_push_packed

    # -- device binding ------------------------------------------------------------
    def _ensure_ctx(self, s, a):
        if self._ctx is None:
            S, A = int(np.asarray(s).size), int(np.asarray(a).size)
            self._ctx = Context(Config(S, A, hidden_dim=4, max_batch=4096, capacity=self.capacity,
                                       replay=self._replay), 0)
        return self._ctx

    @property
    def context(self) -> Context | None:
        return self._ctx

    def _flush(self):
        if not self._rows:
            return
        ctx = self._ctx
        S, A = ctx.cfg.state_dim, ctx.cfg.action_dim
        n = len(self._rows)
        # packed rows s | a | r | s2 | d in a reused buffer (sacmi_push_packed)
        w = 2 * S + A + 2
        if self._pack is None or self._pack.shape[0] < n:
            self._pack = np.empty((max(n, _STAGE), w), np.float32)
        p = self._pack
        for i, (si, ai, ri, s2i, di) in enumerate(self._rows):
            p[i, :S] = np.asarray(si, np.float32).reshape(S)
            p[i, S:S + A] = np.asarray(ai, np.float32).reshape(A)
            p[i, S + A] = ri
            p[i, S + A + 1:w - 1] = np.asarray(s2i, np.float32).reshape(S)
            p[i, w - 1] = 1.0 if di else 0.0
        self._rows.clear()
        ctx.push_packed(p, n)

    def push(self, state, action, reward, next_state, done):
        self._ensure_ctx(state, action)
        self._rows.append((state, action, reward, next_state, done))
        if len(self._rows) >= _STAGE:
            self._flush()

    def __len__(self):
        if self._ctx is None:
            return 0
        return min(self.capacity, len(self._ctx) + len(self._rows))

    def _rows_at(self, idx):
        self._flush()
        return self._ctx.get_rows(np.asarray(idx, np.int64))

    @property
    def buffer(self):
        """Materialised contents (oldest first), as the reference's deque/list of
        5-tuples — used by checkpointing (sac_imp.py:199)."""
        n = len(self)
        if n == 0:
            return deque(maxlen=self.capacity) if self._replay == "uniform" else []
        s, a, r, s2, d = self._rows_at(np.arange(n))
        rows = [(s[i], a[i], float(r[i]), s2[i], bool(d[i])) for i in range(n)]
        return deque(rows, maxlen=self.capacity) if self._replay == "uniform" else rows

    @buffer.setter
    def buffer(self, rows):
        """``buffer = rows`` REPLACES the contents, as the reference's attribute assignment
        does (sac_imp.py:229-230): the ring is emptied, then the rows are pushed in order
        (a deque(maxlen) keeps the last `capacity` of them)."""
        rows = list(rows)
        self._rows.clear()
        if self._ctx is None:
            if not rows:
                return
            self._ensure_ctx(rows[0][0], rows[0][1])
        self._ctx.replay_clear()
        for row in rows:
            self.push(*row)
        self._flush()

    def _replace_arrays(self, s, a, r, s2, d):
        """Replace the contents with the rows of stacked arrays (the drop-in's checkpoint form)."""
        self._rows.clear()
        if len(s) == 0:
            # an empty replay (the reference assigns an empty buffer): nothing to push, and
            # no context to create from rows that do not exist
            if self._ctx is not None:
                self._ctx.replay_clear()
            return
        self._ensure_ctx(s[0], a[0])
        self._ctx.replay_clear()
        self._ctx.push(s, a, r, s2, d)


class ReplayBuffer(_Staged):
    """Uniform replay: push / sample / __len__ / buffer (replay_buffer.py:5-22)."""

    def __init__(self, capacity: int = 1000000, *, ctx: Context | None = None,
                 sync_python_random: bool = True):
        super().__init__(capacity, ctx, "uniform")
        self.sync_python_random = sync_python_random

    def sample_indices(self, batch_size: int) -> np.ndarray:
        self._flush()
        n = len(self)
        if not 0 <= batch_size <= n:
            raise ValueError("Sample larger than population or is negative")
        ctx = self._ctx
        if self.sync_python_random:
            st = random.getstate()
            ctx.set_mt(0, np.array(st[1][:624], np.uint32), st[1][624])
            idx = ctx.sample_indices(batch_size)
            key, pos = ctx.get_mt(0)
            random.setstate((3, tuple(int(x) for x in key) + (pos,), st[2]))
            return idx
        return ctx.sample_indices(batch_size)

    def sample(self, batch_size: int):
        if self._ctx is None:
            raise ValueError("Sample larger than population or is negative")
        idx = self.sample_indices(batch_size)
        s, a, r, s2, d = self._rows_at(idx)
        return (s.astype(np.float64), a, r.astype(np.float64), s2.astype(np.float64), d)


class PrioritizedReplayBuffer(_Staged):
    """Prioritized replay (replay_buffer.py:25-90) on the GPU."""

    def __init__(self, capacity, alpha=0.6, beta_start=0.4, beta_frames=100000, *,
                 ctx: Context | None = None, sync_numpy_random: bool = True):
        super().__init__(capacity, ctx, "per")
        self.alpha = alpha
        self.beta_start = beta_start
        self.beta_frames = beta_frames
        self.sync_numpy_random = sync_numpy_random
        if ctx is not None and ctx.cfg.replay != "per":
            raise ValueError("context was not created with replay='per'")

    def _ensure_ctx(self, s, a):
        if self._ctx is None:
            S, A = int(np.asarray(s).size), int(np.asarray(a).size)
            self._ctx = Context(Config(S, A, hidden_dim=4, max_batch=4096, capacity=self.capacity,
                                       replay="per", per_alpha=self.alpha,
                                       per_beta_start=self.beta_start,
                                       per_beta_frames=self.beta_frames), 0)
        return self._ctx

    @property
    def frame(self) -> int:
        from ._lib import S_PER_FRAME
        return int(self._ctx.get_scalar(S_PER_FRAME)) if self._ctx else 1

    @property
    def priorities(self) -> np.ndarray:
        self._flush()
        if self._ctx is None:
            return np.zeros(self.capacity, np.float32)
        return self._ctx.per_priorities()

    def sample_indices(self, batch_size: int):
        self._flush()
        ctx = self._ctx
        if ctx is None or len(ctx) == 0:
            raise ValueError("probabilities do not sum to 1")
        if self.sync_numpy_random:
            st = np.random.get_state()
            ctx.set_mt(1, st[1], st[2])
            idx, w = ctx.per_sample(batch_size)
            key, pos = ctx.get_mt(1)
            np.random.set_state(("MT19937", key, pos, st[3], st[4]))
            return idx, w
        return ctx.per_sample(batch_size)

    def sample(self, batch_size):
        idx, w = self.sample_indices(batch_size)
        s, a, r, s2, d = self._ctx.get_slots(idx)
        return s, a, r, s2, d.astype(np.float32), idx, w

    def update_priorities(self, indices, priorities):
        self._flush()
        pr = np.array([float(p.item() if hasattr(p, "item") else p) for p in priorities],
                      np.float64)
        # reference: float(p) + 1e-6 in double, stored as float32 (replay_buffer.py:87)
        self._ctx.per_update(np.asarray(indices, np.int64), (pr + 1e-6).astype(np.float32))
