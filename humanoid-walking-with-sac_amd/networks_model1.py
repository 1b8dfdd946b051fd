"""Drop-in for the reference's ``networks_model1`` module (host-side mirrors)."""
from sacmi.networks import GaussianPolicy, QNetwork  # noqa: F401

__all__ = ["QNetwork", "GaussianPolicy"]
