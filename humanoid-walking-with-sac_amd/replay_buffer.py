"""Drop-in for the reference's ``replay_buffer`` module (HBM-resident buffers)."""
from sacmi.replay import PrioritizedReplayBuffer, ReplayBuffer  # noqa: F401

__all__ = ["ReplayBuffer", "PrioritizedReplayBuffer"]
