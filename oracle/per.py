"""numpy restatement of the reference's PrioritizedReplayBuffer arithmetic.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Reference: ``replay_buffer.py:25-90`` (PrioritizedReplayBuffer) and numpy 2.2's
legacy ``RandomState.choice(a, size, p=...)`` which it calls at ``:67``:
``cdf = float64(p).cumsum(); cdf /= cdf[-1]; u = random_sample(size);
idx = cdf.searchsorted(u, side='right')``.

``pairwise_sum_f32`` restates numpy's float32 pairwise summation (the tree behind
``probs.sum()`` at ``:64``) so the HIP kernel's reduction order can be checked
against it bit for bit.
"""
from __future__ import annotations

import numpy as np

from .pyrandom import MT19937

PW_BLOCKSIZE = 128
NPY_BUFSIZE = 8192


def _pairwise(a: np.ndarray) -> np.float32:
    """numpy/_core/src/umath/loops_utils.h.src  @TYPE@_pairwise_sum (float32)."""
    n = a.shape[0]
    f = np.float32
    if n < 8:
        res = f(0.0)   # numpy starts this branch from -0.0 / 0.0; identical for sums
        for i in range(n):
            res = f(res + a[i])
        return res
    if n <= PW_BLOCKSIZE:
        r = [f(a[i]) for i in range(8)]
        i = 8
        while i < n - (n % 8):
            for j in range(8):
                r[j] = f(r[j] + a[i + j])
            i += 8
        res = f(f(f(r[0] + r[1]) + f(r[2] + r[3])) + f(f(r[4] + r[5]) + f(r[6] + r[7])))
        while i < n:
            res = f(res + a[i])
            i += 1
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return f(_pairwise(a[:n2]) + _pairwise(a[n2:]))


def pairwise_sum_f32(a: np.ndarray) -> np.float32:
    """``a.sum()`` for a contiguous 1-D float32 array, as numpy 2.2 computes it: the
    reduction walks the array in NPY_BUFSIZE (8192-element) chunks, sums each chunk
    with the pairwise tree above and adds the chunk sums sequentially (verified
    against ``ndarray.sum`` for n up to 1e6 in tests/test_oracle.py)."""
    a = np.ascontiguousarray(a, dtype=np.float32)
    acc = np.float32(-0.0)
    for c in range(0, a.shape[0], NPY_BUFSIZE):
        acc = np.float32(acc + _pairwise(a[c:c + NPY_BUFSIZE]))
    return acc


def beta_at(frame: int, beta_start=0.4, beta_frames=100000) -> float:
    """replay_buffer.py:54."""
    return min(1.0, beta_start + frame * (1.0 - beta_start) / beta_frames)


def probs_from(prios: np.ndarray, n: int, alpha=0.6) -> np.ndarray:
    """replay_buffer.py:58-64 (float32 pow and float32 normalise)."""
    p = prios[:n] ** alpha
    p /= p.sum()
    return p


def sample_from_probs(probs: np.ndarray, batch: int, mt: MT19937, beta: float):
    """(probs, MT state) -> (indices, weights): np.random.choice + replay_buffer.py:67-71."""
    n = probs.shape[0]
    k = min(batch, n)
    cdf = probs.astype(np.float64).cumsum()
    cdf /= cdf[-1]
    u = np.array([mt.random_sample() for _ in range(k)], dtype=np.float64)
    idx = cdf.searchsorted(u, side="right").astype(np.int64)
    w = (n * probs[idx]) ** (-beta)
    w /= w.max()
    return idx, w.astype(np.float32)


def update_priorities(prios: np.ndarray, idx, new) -> np.ndarray:
    """replay_buffer.py:84-87: sequential, last duplicate wins, +1e-6 in double."""
    out = prios.copy()
    for i, p in zip(idx, new):
        out[int(i)] = np.float32(float(p) + 1e-6)
    return out


def push_priority(prios: np.ndarray, length: int, pos: int, capacity: int):
    """replay_buffer.py:36-46: new entry gets max over the WHOLE array (or 1.0)."""
    out = prios.copy()
    out[pos] = out.max() if length > 0 else np.float32(1.0)
    return out, (pos + 1) % capacity, min(length + 1, capacity)
