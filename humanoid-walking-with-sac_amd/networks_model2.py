"""Drop-in for the reference's ``networks_model2`` module (host-side mirrors of the
3-hidden-layer nets; the SAC drop-in trains them with ``SAC(..., networks="model2")``)."""
from sacmi.networks import GaussianPolicy2 as GaussianPolicy  # noqa: F401
from sacmi.networks import QNetwork2 as QNetwork  # noqa: F401

__all__ = ["QNetwork", "GaussianPolicy"]
