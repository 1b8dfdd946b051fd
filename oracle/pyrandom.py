"""Exact restatement of the integer RNG paths the replay sample depends on.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

* MT19937 as used by CPython's ``_random`` module and by numpy's legacy
  ``RandomState`` (same generator, same tempering).
* ``Random._randbelow_with_getrandbits`` — /usr/lib/python3.10/random.py:239-249.
* ``Random.sample`` (both the pool branch and the set branch) —
  /usr/lib/python3.10/random.py:485-504, called by the reference at
  ``replay_buffer.py:15`` (``random.sample(self.buffer, batch_size)``).  On a deque
  the draws depend only on ``len`` and ``k``, so sampling ``range(n)`` yields the
  deque positions.
* numpy legacy ``random_sample`` (53-bit double from two words), consumed by
  ``np.random.choice`` at ``replay_buffer.py:67``.
"""
from __future__ import annotations

import math

import numpy as np

N = 624
M = 397
MATRIX_A = 0x9908B0DF
UPPER = 0x80000000
LOWER = 0x7FFFFFFF


class MT19937:
    """MT19937 state: 624 key words + position (== CPython's ``index``)."""

    def __init__(self, key, pos: int):
        self.key = np.array(key, dtype=np.uint32).copy()
        assert self.key.shape == (N,)
        self.pos = int(pos)

    # -- state bridges -------------------------------------------------------
    @classmethod
    def from_pystate(cls, state) -> "MT19937":
        """``random.getstate()`` -> (3, (k0..k623, index), gauss_next)."""
        version, internal, _gauss = state
        assert version == 3
        return cls(internal[:N], internal[N])

    def to_pystate(self, gauss_next=None):
        return (3, tuple(int(x) for x in self.key) + (self.pos,), gauss_next)

    @classmethod
    def from_npstate(cls, state) -> "MT19937":
        """``np.random.get_state()`` -> ('MT19937', keys, pos, has_gauss, gauss)."""
        name, keys, pos = state[0], state[1], state[2]
        assert name == "MT19937"
        return cls(keys, pos)

    def to_npstate(self):
        return ("MT19937", self.key.copy(), self.pos, 0, 0.0)

    def copy(self) -> "MT19937":
        return MT19937(self.key, self.pos)

    # -- generator -----------------------------------------------------------
    def twist(self) -> None:
        mt = [int(x) for x in self.key]
        for i in range(N):
            y = (mt[i] & UPPER) | (mt[(i + 1) % N] & LOWER)
            v = mt[(i + M) % N] ^ (y >> 1)
            if y & 1:
                v ^= MATRIX_A
            mt[i] = v
        self.key = np.array(mt, dtype=np.uint32)
        self.pos = 0

    def next_u32(self) -> int:
        if self.pos >= N:
            self.twist()
        y = int(self.key[self.pos])
        self.pos += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y & 0xFFFFFFFF

    def getrandbits(self, k: int) -> int:
        assert 0 < k <= 32, "only k<=32 is on the replay path"
        return self.next_u32() >> (32 - k)

    def randbelow(self, n: int) -> int:
        """random.py:239-249 (_randbelow_with_getrandbits)."""
        if not n:
            return 0
        k = n.bit_length()
        r = self.getrandbits(k)
        while r >= n:
            r = self.getrandbits(k)
        return r

    def random_sample(self) -> float:
        """numpy legacy double: ((a>>5)*2^26 + (b>>6)) / 2^53."""
        a = self.next_u32() >> 5
        b = self.next_u32() >> 6
        return (a * 67108864.0 + b) / 9007199254740992.0


def sample_setsize(k: int) -> int:
    """random.py:488-490 — the pool/set branch threshold (float log, as CPython)."""
    setsize = 21
    if k > 5:
        setsize += 4 ** math.ceil(math.log(k * 3, 4))
    return setsize


def sample_indices(mt: MT19937, n: int, k: int) -> np.ndarray:
    """random.sample(range(n), k) with the given generator; advances ``mt``.

    Raises ValueError exactly like random.py:484-485.
    """
    if not 0 <= k <= n:
        raise ValueError("Sample larger than population or is negative")
    out = np.empty(k, dtype=np.int64)
    if n <= sample_setsize(k):
        pool = list(range(n))
        for i in range(k):
            j = mt.randbelow(n - i)
            out[i] = pool[j]
            pool[j] = pool[n - i - 1]
    else:
        selected = set()
        for i in range(k):
            j = mt.randbelow(n)
            while j in selected:
                j = mt.randbelow(n)
            selected.add(j)
            out[i] = j
    return out


def random_samples(mt: MT19937, count: int) -> np.ndarray:
    return np.array([mt.random_sample() for _ in range(count)], dtype=np.float64)
