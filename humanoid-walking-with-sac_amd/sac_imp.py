"""Drop-in for the reference's ``sac_imp`` module: ``from sac_imp import SAC``.

Put ``humanoid-walking-with-sac_amd/`` on ``sys.path`` (ahead of the reference) and
the reference's trainer.py / main*.py run unchanged with the update on the GPU.
"""
from sacmi.agent import SAC  # noqa: F401

__all__ = ["SAC"]
