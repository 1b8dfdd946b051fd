"""sacmi — MI355X-native SAC gradient step (host side of libsacmi.so).

Public surface mirrors the reference (FilippoCrc/Humanoid-walking-with-SAC):
``SAC`` (sac_imp.py), ``ReplayBuffer`` / ``PrioritizedReplayBuffer``
(replay_buffer.py), ``QNetwork`` / ``GaussianPolicy`` (networks_model1.py).
"""
from .core import Config, Context, setsize  # noqa: F401
from . import _lib  # noqa: F401

__all__ = ["Config", "Context", "setsize"]

from .agent import SAC  # noqa: E402,F401
from .networks import GaussianPolicy, QNetwork  # noqa: E402,F401
from .replay import PrioritizedReplayBuffer, ReplayBuffer  # noqa: E402,F401

__all__ += ["SAC", "ReplayBuffer", "PrioritizedReplayBuffer", "QNetwork", "GaussianPolicy"]
