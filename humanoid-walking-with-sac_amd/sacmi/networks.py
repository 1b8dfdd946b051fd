"""Host-side mirrors of the reference's networks (networks_model1.py, networks_model2.py).

The device owns the live parameters (libsacmi arenas).  These torch modules exist for
what the reference's users do with ``agent.policy`` / ``agent.q1`` ...:

* initialisation — built layer by layer in the reference's order with the same init
  calls (nn.Linear construction, then xavier_uniform_ weights / zero biases), so a
  given ``torch.manual_seed`` yields the reference's initial weights
  (networks_model1.py:11-25,40-63);
* ``state_dict()`` / ``load_state_dict()`` — the checkpoint format of
  sac_imp.py:154-233 (keys ``fc1.weight`` ...); a module bound to a context pushes
  loaded tensors to the device;
* ``forward`` / ``sample`` on CPU for inspection (the training path never uses them).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

LOG_STD_MIN, LOG_STD_MAX = -20, 2


def _xavier_zero(m: nn.Module) -> None:
    if isinstance(m, nn.Linear):
        nn.init.xavier_uniform_(m.weight)
        nn.init.constant_(m.bias, 0)


def _orthogonal_zero(m: nn.Module) -> None:
    """networks_model2.py:72-83 (the policy of model2)."""
    if isinstance(m, nn.Linear):
        nn.init.orthogonal_(m.weight, gain=1.0)
        nn.init.constant_(m.bias, 0.0)


class _DeviceMirror:
    """Mixin: keeps a torch module in sync with one network of a libsacmi context."""

    _sacmi_ctx = None
    _sacmi_net = None

    def bind(self, ctx, net: str, push: bool = True):
        object.__setattr__(self, "_sacmi_ctx", ctx)
        object.__setattr__(self, "_sacmi_net", net)
        if push:
            self.push()
        return self

    def push(self) -> None:
        if self._sacmi_ctx is not None:
            self._sacmi_ctx.set_net(self._sacmi_net, {k: v.detach().cpu().numpy()
                                                      for k, v in self.state_dict().items()})

    def pull(self) -> None:
        if self._sacmi_ctx is None:
            return
        live = self._sacmi_ctx.get_net(self._sacmi_net)
        with torch.no_grad():
            for k, v in nn.Module.state_dict(self).items():
                v.copy_(torch.from_numpy(np.asarray(live[k]).reshape(v.shape)))

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        out = nn.Module.load_state_dict(self, state_dict, strict=strict, assign=assign)
        self.push()
        return out


class _HiddenStack:
    """forward through fc1..fc{n_hidden} with relu."""

    n_hidden = 2

    def _trunk(self, x):
        for i in range(1, self.n_hidden + 1):
            x = F.relu(getattr(self, f"fc{i}")(x))
        return x


class QNetwork(_HiddenStack, _DeviceMirror, nn.Module):
    """Q(s, a): cat -> Linear(S+A,H) relu -> Linear(H,H) relu -> Linear(H,1)."""

    def __init__(self, state_dim: int, action_dim: int, hidden_dim: int = 256):
        nn.Module.__init__(self)
        self.fc1 = nn.Linear(state_dim + action_dim, hidden_dim)
        self.fc2 = nn.Linear(hidden_dim, hidden_dim)
        self.fc3 = nn.Linear(hidden_dim, 1)
        self.apply(_xavier_zero)

    def forward(self, state, action):
        h = self._trunk(torch.cat([state, action], dim=-1))
        return getattr(self, f"fc{self.n_hidden + 1}")(h)


class GaussianPolicy(_HiddenStack, _DeviceMirror, nn.Module):
    """tanh-squashed Gaussian policy with mean / log_std heads."""

    def __init__(self, state_dim: int, action_dim: int, hidden_dim: int = 256,
                 action_bounds=None):
        nn.Module.__init__(self)
        self.fc1 = nn.Linear(state_dim, hidden_dim)
        self.fc2 = nn.Linear(hidden_dim, hidden_dim)
        self.mean = nn.Linear(hidden_dim, action_dim)
        self.log_std = nn.Linear(hidden_dim, action_dim)
        lo, hi = action_bounds if action_bounds is not None else (-0.4, 0.4)
        self.action_scale = (hi - lo) / 2
        self.action_bias = (hi + lo) / 2
        self.apply(_xavier_zero)

    def forward(self, state):
        h = self._trunk(state)
        return self.mean(h), torch.clamp(self.log_std(h), LOG_STD_MIN, LOG_STD_MAX)

    def sample(self, state):
        mean, log_std = self.forward(state)
        std = log_std.exp()
        dist = torch.distributions.Normal(mean, std)
        x = dist.rsample()
        y = torch.tanh(x)
        logp = dist.log_prob(x) - torch.log(self.action_scale * (1 - y.pow(2)) + 1e-6)
        return y * self.action_scale + self.action_bias, logp.sum(dim=-1, keepdim=True)


class QNetwork2(QNetwork):
    """networks_model2.QNetwork (networks_model2.py:18-48): three hidden layers
    fc1..fc3 and the head fc4, xavier-uniform weights, zero biases, default H=512."""

    n_hidden = 3

    def __init__(self, state_dim: int, action_dim: int, hidden_dim: int = 512):
        nn.Module.__init__(self)
        self.fc1 = nn.Linear(state_dim + action_dim, hidden_dim)
        self.fc2 = nn.Linear(hidden_dim, hidden_dim)
        self.fc3 = nn.Linear(hidden_dim, hidden_dim)
        self.fc4 = nn.Linear(hidden_dim, 1)
        self.apply(_xavier_zero)


class GaussianPolicy2(GaussianPolicy):
    """networks_model2.GaussianPolicy (networks_model2.py:51-120): fc1..fc3 + mean /
    log_std heads, orthogonal weights (gain 1), zero biases, default H=512.  ``device``
    is accepted for signature parity; the mirror stays on the host (the live weights are
    in HBM)."""

    n_hidden = 3

    def __init__(self, state_dim: int, action_dim: int, hidden_dim: int = 512, device=None,
                 action_bounds=None):
        nn.Module.__init__(self)
        self.device = device
        self.fc1 = nn.Linear(state_dim, hidden_dim)
        self.fc2 = nn.Linear(hidden_dim, hidden_dim)
        self.fc3 = nn.Linear(hidden_dim, hidden_dim)
        self.mean = nn.Linear(hidden_dim, action_dim)
        self.log_std = nn.Linear(hidden_dim, action_dim)
        lo, hi = action_bounds if action_bounds is not None else (-0.4, 0.4)
        self.action_scale = (hi - lo) / 2
        self.action_bias = (hi + lo) / 2
        self.apply(_orthogonal_zero)


MODELS = {"model1": (QNetwork, GaussianPolicy), "model2": (QNetwork2, GaussianPolicy2)}
