"""Host-side logic of the drop-in that needs no device (CPU tests)."""
import os
import sys
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "humanoid-walking-with-sac_amd"))

from sacmi.agent import SAC  # noqa: E402
from sacmi.replay import PrioritizedReplayBuffer, ReplayBuffer  # noqa: E402


class _FakeCtx:
    """Records the calls a replay restore makes on its context."""

    def __init__(self):
        self.calls = []

    def replay_clear(self):
        self.calls.append("clear")

    def push(self, *rows):
        self.calls.append(("push", len(rows[0])))

    def __len__(self):
        return 0


def _rows_of(rb, S=5, A=2):
    fake = types.SimpleNamespace(_cfg=types.SimpleNamespace(state_dim=S, action_dim=A))
    return SAC._checkpoint_rows(fake, rb)


def test_checkpoint_rows_empty_forms():
    # the reference's empty deque (sac_imp.py:229-230 assigns it) and the drop-in's
    # zero-row tensors both give zero-length arrays of the agent's widths
    for rb in ([], {"state": torch.zeros(0, 5), "action": torch.zeros(0, 2), "reward": torch.zeros(0),
                    "next_state": torch.zeros(0, 5), "done": torch.zeros(0, dtype=torch.bool)}):
        s, a, r, s2, d = _rows_of(rb)
        assert s.shape == (0, 5) and a.shape == (0, 2) and r.shape == (0,) and s2.shape == (0, 5)
        assert d.shape == (0,) and d.dtype == bool


def test_empty_replay_restore_without_context():
    # no context yet: restoring an empty replay creates none and leaves the buffer empty
    for cls in (ReplayBuffer, PrioritizedReplayBuffer):
        rb = cls(100)
        rb._replace_arrays(*_rows_of([]))
        assert rb.context is None and len(rb) == 0


def test_empty_replay_restore_clears_existing_context():
    rb = ReplayBuffer(100)
    ctx = _FakeCtx()
    rb._ctx = ctx
    rb._rows.append((np.zeros(5), np.zeros(2), 0.0, np.zeros(5), False))   # a staged row
    rb._replace_arrays(*_rows_of([]))
    assert ctx.calls == ["clear"] and rb._rows == []


def test_nonempty_replay_restore_pushes_rows():
    rb = ReplayBuffer(100)
    ctx = _FakeCtx()
    rb._ctx = ctx
    rows = [(np.ones(5), np.ones(2), 1.0, np.ones(5), True)] * 3
    rb._replace_arrays(*_rows_of(rows))
    assert ctx.calls == ["clear", ("push", 3)]
