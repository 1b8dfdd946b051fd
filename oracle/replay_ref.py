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
