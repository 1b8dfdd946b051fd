"""Reference-shaped uniform replay for the CPU baseline — TEST/BENCH INFRASTRUCTURE.

Same data path as ``replay_buffer.py:5-22``: a ``deque(maxlen=capacity)`` of 5-tuples
holding references to the caller's arrays, ``random.sample`` over the deque (O(n)
deque indexing), ``zip(*)`` and ``np.array`` stacking.  Used only by bench.py's
``cpu_baseline`` leg to time the reference's CPU update on the GPU box's host.
"""
from __future__ import annotations

import random
from collections import deque

import numpy as np


class DequeReplay:
    def __init__(self, capacity: int = 1_000_000):
        self.rows = deque(maxlen=capacity)

    def push(self, s, a, r, s2, d):
        self.rows.append((s, a, r, s2, d))

    def __len__(self):
        return len(self.rows)

    def sample(self, batch: int):
        picked = random.sample(self.rows, batch)
        cols = list(zip(*picked))
        return tuple(np.array(c) for c in cols)


class PerReplayNumpy:
    """Reference-shaped prioritized replay (``replay_buffer.py:25-87``) for the CPU
    baseline: float32 priority array, max-priority on push, ``prios**alpha`` normalised,
    ``np.random.choice(len, batch, p=probs)``, IS weights ``(N*P)^-beta / max``, rows
    gathered from a list, ``update_priorities`` loop.  Timing port only."""

    def __init__(self, capacity: int = 1_000_000, alpha=0.6, beta_start=0.4, beta_frames=100000):
        self.capacity, self.alpha = capacity, alpha
        self.beta_start, self.beta_frames = beta_start, beta_frames
        self.buffer = []
        self.pos = 0
        self.frame = 1
        self.priorities = np.zeros((capacity,), dtype=np.float32)

    def push(self, s, a, r, s2, d):
        max_prio = self.priorities.max() if self.buffer else 1.0
        if len(self.buffer) < self.capacity:
            self.buffer.append((s, a, r, s2, d))
        else:
            self.buffer[self.pos] = (s, a, r, s2, d)
        self.priorities[self.pos] = max_prio
        self.pos = (self.pos + 1) % self.capacity

    def fill(self, rows):
        """n pushes from empty, in bulk: the state push() leaves (every priority 1.0 —
        the max over a still-all-ones array) without its O(n) max per push."""
        s, a, r, s2, d = rows
        n = min(len(r), self.capacity)
        self.buffer = [(s[i], a[i], float(r[i]), s2[i], bool(d[i])) for i in range(n)]
        self.priorities[:n] = 1.0
        self.pos = n % self.capacity

    def __len__(self):
        return len(self.buffer)

    def sample(self, batch: int):
        n = len(self.buffer)
        beta = min(1.0, self.beta_start + self.frame * (1.0 - self.beta_start) / self.beta_frames)
        self.frame += 1
        probs = self.priorities[:n] ** self.alpha
        probs /= probs.sum()
        idx = np.random.choice(n, batch, p=probs)
        cols = list(zip(*[self.buffer[i] for i in idx]))
        w = (n * probs[idx]) ** (-beta)
        w /= w.max()
        return tuple(np.array(c) for c in cols) + (idx, np.array(w, dtype=np.float32))

    def update_priorities(self, idx, prios):
        for i, p in zip(idx, prios):
            self.priorities[i] = p + 1e-6
