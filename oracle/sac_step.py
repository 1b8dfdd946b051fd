"""Functional torch-CPU restatement of one SAC gradient step.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Follows the reference op for op so that, in float32 with the same minibatch and the
same Gaussian noise, it reproduces the reference bit for bit (checked against
``tests/golden/step_small.npz`` in ``tests/test_oracle.py``); in float64 it is the
high-precision truth the HIP path is graded against.

Reference map
-------------
* QNetwork.forward            networks_model1.py:27-33   (cat -> fc1 relu fc2 relu fc3)
                              networks_model2.py:37-48   (n_hidden=3: ... fc3 relu fc4)
* GaussianPolicy.forward      networks_model1.py:65-76   (log_std clamp [-20, 2])
                              networks_model2.py:86-99   (n_hidden=3: fc1 fc2 fc3, heads)
* GaussianPolicy.sample       networks_model1.py:78-99   (rsample, tanh squash, log-prob)
* SAC.update_parameters       sac_imp.py:74-144
* SAC._soft_update_target...  sac_imp.py:146-152
* Adam (torch.optim, single-tensor, CPU)  — same library the reference calls at
  sac_imp.py:39-41,49.

Noise is injected: ``eps1`` replaces the ``normal_()`` draw inside
``policy.sample(next_state_batch)`` (sac_imp.py:89) and ``eps2`` the one inside
``policy.sample(state_batch)`` (sac_imp.py:116); nothing else in the step consumes
torch RNG.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import torch
import torch.nn.functional as F

POLICY_KEYS = ("fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias",
               "mean.weight", "mean.bias", "log_std.weight", "log_std.bias")
Q_KEYS = ("fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias", "fc3.weight", "fc3.bias")


def policy_keys(n_hidden: int = 2) -> tuple:
    """state_dict keys of GaussianPolicy: networks_model1.py:46-50 (2 hidden layers),
    networks_model2.py:57-62 (3)."""
    hid = tuple(f"fc{i}.{p}" for i in range(1, n_hidden + 1) for p in ("weight", "bias"))
    return hid + POLICY_KEYS[4:]


def q_keys(n_hidden: int = 2) -> tuple:
    """state_dict keys of QNetwork: networks_model1.py:14-17 (fc1..fc3), model2 :23-27
    (fc1..fc4)."""
    return tuple(f"fc{i}.{p}" for i in range(1, n_hidden + 2) for p in ("weight", "bias"))


NETS = ("policy", "q1", "q2", "q1_target", "q2_target")


@dataclass
class SacConfig:
    state_dim: int
    action_dim: int
    hidden_dim: int = 256
    gamma: float = 0.99
    tau: float = 0.005
    lr: float = 3e-4
    alpha: float = 0.2
    automatic_entropy_tuning: bool = True
    action_low: float = -0.4
    action_high: float = 0.4
    n_hidden: int = 2          # 2: networks_model1 (the reference's SAC), 3: networks_model2

    @property
    def action_scale(self) -> float:   # networks_model1.py:54
        return (self.action_high - self.action_low) / 2

    @property
    def action_bias(self) -> float:    # networks_model1.py:55
        return (self.action_high + self.action_low) / 2


def param_shapes(cfg: SacConfig) -> dict:
    S, A, H, nh = cfg.state_dim, cfg.action_dim, cfg.hidden_dim, cfg.n_hidden
    pol = {"fc1.weight": (H, S), "fc1.bias": (H,)}
    for i in range(2, nh + 1):
        pol.update({f"fc{i}.weight": (H, H), f"fc{i}.bias": (H,)})
    pol.update({"mean.weight": (A, H), "mean.bias": (A,), "log_std.weight": (A, H),
                "log_std.bias": (A,)})
    q = {"fc1.weight": (H, S + A), "fc1.bias": (H,)}
    for i in range(2, nh + 1):
        q.update({f"fc{i}.weight": (H, H), f"fc{i}.bias": (H,)})
    q.update({f"fc{nh + 1}.weight": (1, H), f"fc{nh + 1}.bias": (1,)})
    return {"policy": pol, "q1": q, "q2": q, "q1_target": q, "q2_target": q}


def orthogonal(rng, shape) -> np.ndarray:
    """Portable stand-in for torch.nn.init.orthogonal_(w, gain=1) (networks_model2.py:82):
    QR of a Gaussian matrix, sign-corrected by diag(R), rows orthonormal when out <= in
    (columns otherwise)."""
    rows, cols = shape
    flat = rng.standard_normal((rows, cols))
    if rows < cols:
        flat = flat.T
    q, r = np.linalg.qr(flat)
    q *= np.sign(np.diag(r))
    if rows < cols:
        q = q.T
    return q.astype(np.float32)


def init_params(cfg: SacConfig, seed: int, bias_scale: float = 0.0) -> dict:
    """Portable (numpy PCG64) stand-in for the reference's xavier_uniform init
    (networks_model1.py:22-25,60-63): W ~ U(-b, b), b = sqrt(6/(fan_in+fan_out));
    with n_hidden=3 the policy weights are orthogonal (networks_model2.py:72-83).
    Biases are 0 as in the reference unless ``bias_scale`` > 0 (tests use non-zero
    biases so the bias gradients are exercised).  Targets copy q1/q2
    (sac_imp.py:33-36)."""
    rng = np.random.default_rng(seed)
    shapes = param_shapes(cfg)
    out = {}
    for net in ("policy", "q1", "q2"):
        d = {}
        for k, shp in shapes[net].items():
            if k.endswith("weight") and net == "policy" and cfg.n_hidden == 3:
                d[k] = orthogonal(rng, shp)
            elif k.endswith("weight"):
                b = math.sqrt(6.0 / (shp[0] + shp[1]))
                d[k] = rng.uniform(-b, b, size=shp).astype(np.float32)
            else:
                d[k] = (rng.uniform(-bias_scale, bias_scale, size=shp).astype(np.float32)
                        if bias_scale > 0 else np.zeros(shp, np.float32))
        out[net] = d
    out["q1_target"] = {k: v.copy() for k, v in out["q1"].items()}
    out["q2_target"] = {k: v.copy() for k, v in out["q2"].items()}
    return out


def synthetic_rows(cfg: SacConfig, n: int, seed: int, state_scale: float = 1.0):
    """Synthetic transitions: s,s2 ~ N(0, scale^2), a ~ U(-0.4,0.4),
    r ~ N(0,1), done ~ Bernoulli(0.02).  float32 / uint8."""
    rng = np.random.default_rng(seed)
    S, A = cfg.state_dim, cfg.action_dim
    s = (rng.standard_normal((n, S)) * state_scale).astype(np.float32)
    a = rng.uniform(cfg.action_low, cfg.action_high, size=(n, A)).astype(np.float32)
    r = rng.standard_normal(n).astype(np.float32)
    s2 = (rng.standard_normal((n, S)) * state_scale).astype(np.float32)
    d = (rng.random(n) < 0.02).astype(np.uint8)
    return s, a, r, s2, d


# ----------------------------------------------------------------------------
def _n_hidden(p) -> int:
    return sum(1 for k in p if k.startswith("fc") and k.endswith(".weight")) - (
        0 if "mean.weight" in p else 1)


# ----------------------------------------------------------------------------
# bf16-operand emulation (test infrastructure for compute_dtype=bf16, which has no
# reference counterpart: BASELINE configs[4]).  Where the HIP path feeds a GEMM's operands
# to a bf16 MFMA, the emulation rounds them to bf16 (round-to-nearest-even) and multiplies
# in the oracle's dtype; the GEMMs the HIP path keeps in fp32 (policy heads forward and
# their dX, the critic head's forward dot and the dL/da product) stay unrounded.  Roles:
#   in   first hidden layer: x = [input | 1] against [W | b] (bias folded into K, so
#        rounded; dW's bias column is the sum of rounded dY); dX unrounded (dL/da)
#   hid  later hidden layers: forward, dX and dW rounded; bias add / bias grad fp32
#   head critic fc{n+1}: forward and dX unrounded (dot epilogue / row transform), dW
#        rounded;  phead: policy mean / log_std, the same
# act (bf16 activations, sacmi_step_act16: batch-4096 class): the HIP path stores every
# activation as bf16, so the policy heads' forward input is the rounded h (straight-through
# for the gradient: their dX stays unrounded); every other operand is rounded as above
# already, and the critic head dots read the unrounded epilogue values.
_ROUND = {"on": False, "act": False}

# Forced ReLU masks (test infrastructure): {(pass tag, hidden layer index): {0,1} tensor of the
# layer's output shape}.  With a mask given, the layer's output is pre * mask instead of
# relu(pre), and its backward is masked the same way: the update evaluated in the oracle's
# precision under ANOTHER evaluation's ReLU decisions (the GPU's: sacmi_read_activation), which
# separates fp32 summation-order flips of near-zero pre-activations from kernel error.
# Tags: q1 / q2 (critics on (s, a)), q1t / q2t (targets on (s', a')), pi_s2 / pi_s (policy on
# s' / s), q1a / q2a (updated critics on (s, a~)).
_MASKS: dict = {}


def _relu(x, tag, i):
    m = _MASKS.get((tag, i)) if tag else None
    return F.relu(x) if m is None else x * m.to(x.dtype)


def _bf(t):
    return t.to(torch.bfloat16).to(t.dtype)


class _EmuLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, role):
        ctx.save_for_backward(x, w)
        ctx.role = role
        if role == "in":
            return _bf(x) @ _bf(w).T + _bf(b)
        if role == "hid":
            return _bf(x) @ _bf(w).T + b
        return x @ w.T + b

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        role = ctx.role
        dx = _bf(g) @ _bf(w) if role == "hid" else g @ w
        dw = _bf(g).T @ _bf(x)
        db = _bf(g).sum(0) if role == "in" else g.sum(0)
        return dx, dw, db, None


def _lin(x, w, b, role):
    if _ROUND["on"]:
        return _EmuLinear.apply(x, w, b, role)
    return F.linear(x, w, b)


def _q_forward(p, state, action, tag=None):
    x = torch.cat([state, action], dim=-1)
    nh = _n_hidden(p)
    for i in range(1, nh + 1):
        x = _relu(_lin(x, p[f"fc{i}.weight"], p[f"fc{i}.bias"], "in" if i == 1 else "hid"), tag, i - 1)
    return _lin(x, p[f"fc{nh + 1}.weight"], p[f"fc{nh + 1}.bias"], "head")


def _policy_forward(p, state, tag=None):
    x = state
    for i in range(1, _n_hidden(p) + 1):
        x = _relu(_lin(x, p[f"fc{i}.weight"], p[f"fc{i}.bias"], "in" if i == 1 else "hid"), tag, i - 1)
    if _ROUND["on"] and _ROUND["act"]:
        x = x + (_bf(x) - x).detach()
    mean = _lin(x, p["mean.weight"], p["mean.bias"], "head")
    log_std = _lin(x, p["log_std.weight"], p["log_std.bias"], "head")
    return mean, torch.clamp(log_std, -20, 2)


def _policy_sample(p, state, eps, scale, bias, tag=None):
    mean, log_std = _policy_forward(p, state, tag)
    std = log_std.exp()
    normal = torch.distributions.Normal(mean, std)
    x_t = mean + eps * std                     # Normal.rsample with injected eps
    y_t = torch.tanh(x_t)
    action = y_t * scale + bias
    log_prob = normal.log_prob(x_t)
    log_prob -= torch.log(scale * (1 - y_t.pow(2)) + 1e-6)
    log_prob = log_prob.sum(dim=-1, keepdim=True)
    return action, log_prob


@dataclass
class OracleSAC:
    """One agent's full training state; ``step`` = one ``update_parameters`` call."""
    cfg: SacConfig
    params: dict                       # net -> key -> np.ndarray
    dtype: torch.dtype = torch.float64
    nets: dict = field(init=False)
    opt: dict = field(init=False)
    log_alpha: torch.Tensor = field(init=False)
    alpha: object = field(init=False)
    last_grads: dict = field(init=False, default_factory=dict)

    def __post_init__(self):
        dt = self.dtype
        self.nets = {n: {k: torch.tensor(np.asarray(v), dtype=dt).requires_grad_(n in ("policy", "q1", "q2"))
                         for k, v in self.params[n].items()} for n in NETS}
        lr = self.cfg.lr
        self.opt = {n: torch.optim.Adam(list(self.nets[n].values()), lr=lr)
                    for n in ("policy", "q1", "q2")}
        self.log_alpha = torch.zeros(1, dtype=dt, requires_grad=True)
        if self.cfg.automatic_entropy_tuning:
            self.opt["alpha"] = torch.optim.Adam([self.log_alpha], lr=lr)
        self.alpha = self.cfg.alpha                     # python float until 1st update

    def step(self, s, a, r, s2, d, eps1, eps2, bf16_operands: bool = False,
             bf16_act: bool = False, masks: dict | None = None) -> dict:
        """``bf16_operands``: emulate compute_dtype=bf16 (see _EmuLinear); ``bf16_act``:
        with bf16-stored activations (sacmi_step_act16); ``masks``: forced ReLU masks
        (see _MASKS: {(tag, layer): array})."""
        _ROUND["on"] = bool(bf16_operands)
        _ROUND["act"] = bool(bf16_act)
        _MASKS.clear()
        for k, m in (masks or {}).items():
            _MASKS[k] = torch.as_tensor(np.asarray(m, dtype=np.float32))
        try:
            return self._step(s, a, r, s2, d, eps1, eps2)
        finally:
            _ROUND["on"] = False
            _ROUND["act"] = False
            _MASKS.clear()

    def _step(self, s, a, r, s2, d, eps1, eps2) -> dict:
        cfg, dt = self.cfg, self.dtype
        T = lambda x: torch.as_tensor(np.asarray(x, dtype=np.float32)).to(dt)
        state, action, next_state = T(s), T(a), T(s2)
        reward = T(r).reshape(-1, 1)
        done = T(d).reshape(-1, 1)
        e1, e2 = T(eps1), T(eps2)
        P, Q1, Q2 = self.nets["policy"], self.nets["q1"], self.nets["q2"]
        sc, bi = cfg.action_scale, cfg.action_bias
        with torch.no_grad():
            na, nlp = _policy_sample(P, next_state, e1, sc, bi, "pi_s2")
            q1n = _q_forward(self.nets["q1_target"], next_state, na, "q1t")
            q2n = _q_forward(self.nets["q2_target"], next_state, na, "q2t")
            value_target = torch.min(q1n, q2n) - self.alpha * nlp
            q_target = reward + (1 - done) * cfg.gamma * value_target
        q1_loss = F.mse_loss(_q_forward(Q1, state, action, "q1"), q_target)
        q2_loss = F.mse_loss(_q_forward(Q2, state, action, "q2"), q_target)
        grads = {}
        self.opt["q1"].zero_grad(); q1_loss.backward()
        grads["q1"] = {k: v.grad.detach().clone() for k, v in Q1.items()}
        self.opt["q1"].step()
        self.opt["q2"].zero_grad(); q2_loss.backward()
        grads["q2"] = {k: v.grad.detach().clone() for k, v in Q2.items()}
        self.opt["q2"].step()

        policy_loss = self._actor(state, e2, grads)
        with torch.no_grad():
            tau = cfg.tau
            for src, dst in (("q1", "q1_target"), ("q2", "q2_target")):
                for k in q_keys(cfg.n_hidden):
                    t = self.nets[dst][k]
                    t.copy_(t * (1.0 - tau) + self.nets[src][k] * tau)
        self.last_grads = grads
        return {"q1_loss": q1_loss.item(), "q2_loss": q2_loss.item(),
                "policy_loss": policy_loss.item()}

    def _actor(self, state, e2, grads):
        """The actor and alpha blocks (sac_imp.py:116-135) on the agent's current critics."""
        cfg = self.cfg
        P, Q1, Q2 = self.nets["policy"], self.nets["q1"], self.nets["q2"]
        new_a, logp = _policy_sample(P, state, e2, cfg.action_scale, cfg.action_bias, "pi_s")
        q_new = torch.min(_q_forward(Q1, state, new_a, "q1a"), _q_forward(Q2, state, new_a, "q2a"))
        policy_loss = (self.alpha * logp - q_new).mean()
        self.opt["policy"].zero_grad(); policy_loss.backward()
        grads["policy"] = {k: v.grad.detach().clone() for k, v in P.items()}
        self.opt["policy"].step()
        if cfg.automatic_entropy_tuning:
            target_entropy = -cfg.action_dim
            alpha_loss = -(self.log_alpha * (logp + target_entropy).detach()).mean()
            self.opt["alpha"].zero_grad(); alpha_loss.backward()
            grads["log_alpha"] = self.log_alpha.grad.detach().clone()
            self.opt["alpha"].step()
            self.alpha = self.log_alpha.exp()
        return policy_loss

    def actor_step(self, s, eps2) -> float:
        """The actor and alpha blocks of one update_parameters call alone (sac_imp.py:116-135),
        on the agent's CURRENT critics: the reference for an update whose critic step happened
        elsewhere (the sharded data-parallel chunk tests load the partly stepped critics)."""
        T = lambda x: torch.as_tensor(np.asarray(x, dtype=np.float32)).to(self.dtype)
        grads = {}
        loss = self._actor(T(s), T(eps2), grads)
        self.last_grads = grads
        return loss.item()

    # -- snapshots ------------------------------------------------------------
    def state(self) -> dict:
        """Flat dict of numpy arrays: '<net>.<key>', 'adam.<net>.<key>.m/v', ..."""
        out = {}
        for n in NETS:
            for k, v in self.nets[n].items():
                out[f"{n}.{k}"] = v.detach().numpy().copy()
        for n in ("policy", "q1", "q2"):
            for k, v in self.nets[n].items():
                st = self.opt[n].state.get(v, {})
                if st:
                    out[f"adam.{n}.{k}.m"] = st["exp_avg"].numpy().copy()
                    out[f"adam.{n}.{k}.v"] = st["exp_avg_sq"].numpy().copy()
                    out[f"adam.{n}.step"] = np.array(float(st["step"]))
        out["log_alpha"] = self.log_alpha.detach().numpy().copy()
        if "alpha" in self.opt and self.opt["alpha"].state.get(self.log_alpha):
            st = self.opt["alpha"].state[self.log_alpha]
            out["adam.log_alpha.m"] = st["exp_avg"].numpy().copy()
            out["adam.log_alpha.v"] = st["exp_avg_sq"].numpy().copy()
        a = self.alpha
        out["alpha"] = np.array(float(a) if not torch.is_tensor(a) else float(a.detach()))
        return out

    def grads_flat(self) -> dict:
        out = {}
        for n, d in self.last_grads.items():
            if isinstance(d, dict):
                for k, v in d.items():
                    out[f"{n}.{k}"] = v.numpy().copy()
            else:
                out[n] = d.numpy().copy()
        return out
