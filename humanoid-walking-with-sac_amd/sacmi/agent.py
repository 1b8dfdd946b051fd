"""Drop-in ``SAC`` (reference sac_imp.py) whose update runs as HIP kernels on one MI355X.

Same constructor arguments, attributes and methods as sac_imp.SAC:
``update_parameters(batch_size)`` (sac_imp.py:74-144), ``select_action``
(:54-72), ``save`` / ``load`` (:154-173), ``save_checkpoint`` / ``load_checkpoint``
(:177-233), and the attributes ``policy, q1, q2, q1_target, q2_target,
*_optimizer, log_alpha, alpha, target_entropy, replay_buffer``.

The live state (parameters, Adam moments, alpha, replay rows) is in HBM; the torch
modules/optimizers are host mirrors refreshed on access after an update and pushed
back on ``load_state_dict``.  There is no CPU fallback: constructing on a machine
without a HIP device raises.
"""
from __future__ import annotations

import random

import numpy as np
import torch

from . import _lib as L
from .core import Config, Context, net_keys
from .networks import MODELS
from .replay import ReplayBuffer

_OPT_NETS = ("policy", "q1", "q2")


def _load_checkpoint_file(path):
    """torch.load with the weights-only unpickler (nothing in the file is executed), plus the
    numpy array / scalar reconstructors on its allowlist so that a replay buffer saved as
    the reference's list of (state, action, reward, next_state, done) tuples of numpy
    values (sac_imp.py:199 with PrioritizedReplayBuffer.buffer, replay_buffer.py:28) loads.
    The uniform buffer's ``deque`` cannot be rebuilt by that unpickler at all: such a
    checkpoint raises, and the buffer must be stored as a list (``list(buffer)``)."""
    try:
        import numpy._core.multiarray as _ma       # numpy >= 2
    except ImportError:                            # pragma: no cover
        import numpy.core.multiarray as _ma
    allow = [_ma._reconstruct, _ma.scalar, np.ndarray, np.dtype]
    allow += [type(np.dtype(t)) for t in (np.float64, np.float32, np.float16, np.int64,
                                          np.int32, np.uint8, np.bool_)]
    with torch.serialization.safe_globals(allow):
        return torch.load(path, weights_only=True, map_location="cpu")


def _device_index(device) -> int:
    if device is None:
        return 0
    if isinstance(device, int):
        return device
    d = torch.device(device)
    if d.type != "cuda":
        raise RuntimeError(f"sacmi runs on a HIP device; got device={device!r} "
                           "(there is no CPU fallback)")
    return d.index or 0


class _AdamMirror(torch.optim.Adam):
    """torch Adam over host mirrors; its state is the device's Adam state."""

    def __init__(self, params, lr, agent, net):
        super().__init__(params, lr=lr)
        self._agent, self._net = agent, net

    def _tensors(self):
        return self.param_groups[0]["params"]

    def _pull(self):
        ctx = self._agent._ctx
        if self._net == "alpha":
            st = ctx.get_scalar(L.S_STEP_ALPHA)
            if st == 0:
                self.state.clear()
                return
            p = self._tensors()[0]
            self.state[p] = {"step": torch.tensor(float(st)),
                             "exp_avg": torch.tensor([ctx.get_scalar(L.S_ADAM_M_LOG_ALPHA)]),
                             "exp_avg_sq": torch.tensor([ctx.get_scalar(L.S_ADAM_V_LOG_ALPHA)])}
            return
        step = ctx.get_scalar({"policy": L.S_STEP_POLICY, "q1": L.S_STEP_Q1,
                               "q2": L.S_STEP_Q2}[self._net])
        if step == 0:
            self.state.clear()
            return
        m = ctx.get_net(self._net, "m")
        v = ctx.get_net(self._net, "v")
        for p, (key, _l, _p) in zip(self._tensors(), net_keys(self._net, self._agent._cfg.n_hidden)):
            self.state[p] = {"step": torch.tensor(float(step)),
                             "exp_avg": torch.from_numpy(m[key].reshape(p.shape)).clone(),
                             "exp_avg_sq": torch.from_numpy(v[key].reshape(p.shape)).clone()}

    def _push(self):
        ctx = self._agent._ctx
        ps = self._tensors()
        st = [self.state.get(p, {}) for p in ps]
        step = float(st[0]["step"]) if st and st[0] else 0.0
        if self._net == "alpha":
            ctx.set_scalar(L.S_STEP_ALPHA, step)
            if st[0]:
                ctx.set_scalar(L.S_ADAM_M_LOG_ALPHA, float(st[0]["exp_avg"].reshape(-1)[0]))
                ctx.set_scalar(L.S_ADAM_V_LOG_ALPHA, float(st[0]["exp_avg_sq"].reshape(-1)[0]))
            return
        which = {"policy": L.S_STEP_POLICY, "q1": L.S_STEP_Q1, "q2": L.S_STEP_Q2}[self._net]
        ctx.set_scalar(which, step)
        if st and st[0]:
            keys = [k for k, _l, _p in net_keys(self._net, self._agent._cfg.n_hidden)]
            ctx.set_net(self._net, {k: s["exp_avg"].numpy() for k, s in zip(keys, st)}, "m")
            ctx.set_net(self._net, {k: s["exp_avg_sq"].numpy() for k, s in zip(keys, st)}, "v")

    def state_dict(self):
        self._agent._flush_device()
        self._pull()
        return super().state_dict()

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        self._push()

    def step(self, closure=None):   # the device owns the optimisation
        raise RuntimeError("sacmi: optimizer steps run on the GPU inside update_parameters()")


class SAC:
    """Soft Actor-Critic for continuous action spaces, MI355X-native update."""

    def __init__(self, state_dim, action_dim, hidden_dim=256, gamma=0.99, tau=0.005, lr=3e-4,
                 alpha=0.2, automatic_entropy_tuning=True, device=None, *,
                 capacity: int = 1000000, max_batch: int = 4096, action_bounds=None,
                 seed: int | None = None, sync_python_random: bool = False,
                 networks: str = "model1", compute_dtype: str = "fp32"):
        """``networks``: "model1" (networks_model1, the reference's import at
        sac_imp.py:4) or "model2" (networks_model2: three hidden layers, orthogonal
        policy init — the swap the reference makes by editing that import).
        ``compute_dtype``: "fp32" (the reference's arithmetic) or "bf16" (bf16 MFMA
        operands with fp32 accumulation, fp32 master weights / Adam / losses)."""
        if networks not in MODELS:
            raise ValueError(f"networks must be one of {sorted(MODELS)}")
        QNetwork, GaussianPolicy = MODELS[networks]
        self.gamma = gamma
        self.tau = tau
        self.device = device if device is not None else "cuda"
        self.automatic_entropy_tuning = automatic_entropy_tuning
        # host mirrors, built exactly in the reference's order (sac_imp.py:28-36)
        policy = GaussianPolicy(state_dim, action_dim, hidden_dim, action_bounds=action_bounds)
        q1 = QNetwork(state_dim, action_dim, hidden_dim)
        q2 = QNetwork(state_dim, action_dim, hidden_dim)
        q1_target = QNetwork(state_dim, action_dim, hidden_dim)
        q2_target = QNetwork(state_dim, action_dim, hidden_dim)
        q1_target.load_state_dict(q1.state_dict())
        q2_target.load_state_dict(q2.state_dict())
        lo, hi = action_bounds if action_bounds is not None else (-0.4, 0.4)
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        self._cfg = Config(state_dim, action_dim, hidden_dim, max_batch=max_batch, gamma=gamma,
                           tau=tau, lr=lr, alpha=float(alpha),
                           automatic_entropy_tuning=automatic_entropy_tuning,
                           action_low=lo, action_high=hi, capacity=capacity, seed=seed,
                           n_hidden=QNetwork.n_hidden, compute_dtype=compute_dtype)
        self._ctx = Context(self._cfg, _device_index(device))
        self._mods = {"policy": policy, "q1": q1, "q2": q2, "q1_target": q1_target,
                      "q2_target": q2_target}
        for name, mod in self._mods.items():
            mod.bind(self._ctx, name)
        self._stale = False
        self.policy_optimizer = _AdamMirror(policy.parameters(), lr, self, "policy")
        self.q1_optimizer = _AdamMirror(q1.parameters(), lr, self, "q1")
        self.q2_optimizer = _AdamMirror(q2.parameters(), lr, self, "q2")
        self._log_alpha = torch.zeros(1, requires_grad=True)
        if automatic_entropy_tuning:
            self.target_entropy = -action_dim
            self.alpha_optimizer = _AdamMirror([self._log_alpha], lr, self, "alpha")
        self.replay_buffer = ReplayBuffer(capacity, ctx=self._ctx,
                                          sync_python_random=sync_python_random)
        st = random.getstate()             # device sampling stream starts at `random`'s
        self._ctx.set_mt(0, np.array(st[1][:624], np.uint32), st[1][624])
        self._mt_adopted = st[1]           # (the Python stream state the device holds)

    # -- mirrored attributes ---------------------------------------------------------
    def _flush_device(self):
        self.replay_buffer._flush()

    def _mirror(self, name):
        if self._stale:
            for m in self._mods.values():
                m.pull()
            with torch.no_grad():
                self._log_alpha.fill_(self._ctx.get_scalar(L.S_LOG_ALPHA))
            self._stale = False
        return self._mods[name]

    policy = property(lambda self: self._mirror("policy"))
    q1 = property(lambda self: self._mirror("q1"))
    q2 = property(lambda self: self._mirror("q2"))
    q1_target = property(lambda self: self._mirror("q1_target"))
    q2_target = property(lambda self: self._mirror("q2_target"))

    @property
    def log_alpha(self):
        self._mirror("policy")
        return self._log_alpha

    @log_alpha.setter
    def log_alpha(self, value):
        v = float(torch.as_tensor(value).detach().reshape(-1)[0])
        with torch.no_grad():
            self._log_alpha.fill_(v)
        self._ctx.set_scalar(L.S_LOG_ALPHA, v)

    @property
    def alpha(self):
        """0.2-style float until the first update, then exp(log_alpha) as a [1] tensor
        (sac_imp.py:22,135)."""
        if self._ctx.get_scalar(L.S_ALPHA_IS_TENSOR):
            return torch.tensor([self._ctx.get_scalar(L.S_ALPHA)], dtype=torch.float32)
        return self._cfg.alpha

    @alpha.setter
    def alpha(self, value):
        if torch.is_tensor(value):
            self._ctx.set_scalar(L.S_ALPHA, float(value.detach().reshape(-1)[0]))
            self._ctx.set_scalar(L.S_ALPHA_IS_TENSOR, 1)
        else:
            self._ctx.set_scalar(L.S_ALPHA, float(value))
            self._ctx.set_scalar(L.S_ALPHA_IS_TENSOR, 0)
            self._cfg.alpha = float(value)

    # -- hot path ----------------------------------------------------------------------
    def update_parameters(self, batch_size=256):
        """One SAC update (sac_imp.py:74-144); returns the three losses as floats."""
        self._flush_device()
        if len(self.replay_buffer) < batch_size:
            raise ValueError("Sample larger than population or is negative")
        rb = self.replay_buffer
        self._stale = True     # (also when it raises: the critic step may have been taken)
        if rb.sync_python_random and batch_size <= 4096 and self._ctx.cfg.replay == "uniform":
            st = random.getstate()
            if st[1] != self._mt_adopted:   # the stream moved (drawn from, seeded): adopt it
                self._ctx.set_mt(0, np.array(st[1][:624], np.uint32), st[1][624])
            self._ctx.step_launch(batch_size)
            try:
                # while the GPU runs the update, the reference's own random.sample
                # (sac_imp.py:75) advances Python's stream: its draws depend only on the
                # population size and k, and the device drew the same indices from the
                # same state (test_sync_python_random_consumes_like_reference)
                random.sample(range(len(rb)), batch_size)
            finally:           # (the sample ran even if the update raises)
                try:
                    out = self._ctx.step_wait()
                finally:
                    self._mt_adopted = random.getstate()[1]
        elif rb.sync_python_random:
            st = random.getstate()
            self._ctx.set_mt(0, np.array(st[1][:624], np.uint32), st[1][624])
            try:
                out = self._ctx.step(batch_size)
            finally:           # the update's random.sample ran even if the update raised
                key, pos = self._ctx.get_mt(0)
                random.setstate((3, tuple(int(x) for x in key) + (pos,), st[2]))
        else:
            out = self._ctx.step(batch_size)
        return {"q1_loss": float(out[0]), "q2_loss": float(out[1]), "policy_loss": float(out[2])}

    def update_parameters_async(self, batch_size=256):
        """Same update, enqueued without a host sync (losses: fetch_losses())."""
        self._flush_device()
        self._ctx.step_async(batch_size)
        self._stale = True

    def update_parameters_many(self, batch_size=256, n_updates=1):
        """The trainer's `for _ in range(updates_per_step): update_parameters(batch_size)`
        (trainer.py:203-204) as one device launch; returns the last update's losses,
        which is what that loop keeps."""
        self._flush_device()
        if len(self.replay_buffer) < batch_size:
            raise ValueError("Sample larger than population or is negative")
        rb = self.replay_buffer
        if rb.sync_python_random:
            st = random.getstate()
            self._ctx.set_mt(0, np.array(st[1][:624], np.uint32), st[1][624])
        self._stale = True
        self._ctx.step_many_async(batch_size, n_updates)
        if rb.sync_python_random:
            key, pos = self._ctx.get_mt(0)
            random.setstate((3, tuple(int(x) for x in key) + (pos,), st[2]))
        # raises ValueError at the first update whose policy sample was NaN (the loop of
        # trainer.py:203-204 stops there; the later updates of the launch took no step)
        out = self._ctx.fetch_losses(1)[0]
        return {"q1_loss": float(out[0]), "q2_loss": float(out[1]), "policy_loss": float(out[2])}

    def fetch_losses(self, max_steps=4096):
        rows = self._ctx.fetch_losses(max_steps)
        return [{"q1_loss": float(r[0]), "q2_loss": float(r[1]), "policy_loss": float(r[2])}
                for r in rows]

    def select_action(self, state, evaluate=False):
        """sac_imp.py:54-72: tanh(mean) when evaluating, a policy sample otherwise."""
        s = np.asarray(state, np.float32)
        single = s.ndim == 1
        a = self._ctx.act(s.reshape(1, -1) if single else s, deterministic=bool(evaluate))
        return a[0] if single else a

    # -- checkpoints (sac_imp.py:154-233) ----------------------------------------------------
    def save(self, path):
        torch.save({"policy_state_dict": self.policy.state_dict(),
                    "q1_state_dict": self.q1.state_dict(),
                    "q2_state_dict": self.q2.state_dict(),
                    "q1_target_state_dict": self.q1_target.state_dict(),
                    "q2_target_state_dict": self.q2_target.state_dict(),
                    "alpha": self.alpha}, path)

    def load(self, path):
        ck = _load_checkpoint_file(path)
        self._load_nets(ck)
        self.alpha = ck["alpha"]

    def _load_nets(self, ck):
        for name in ("policy", "q1", "q2", "q1_target", "q2_target"):
            self._mirror(name).load_state_dict(ck[f"{name}_state_dict"])

    def save_checkpoint(self, path, episode, total_steps, replay_buffer=True):
        ck = {"episode": episode, "total_steps": total_steps,
              "policy_state_dict": self.policy.state_dict(),
              "q1_state_dict": self.q1.state_dict(), "q2_state_dict": self.q2.state_dict(),
              "q1_target_state_dict": self.q1_target.state_dict(),
              "q2_target_state_dict": self.q2_target.state_dict(),
              "policy_optimizer_state_dict": self.policy_optimizer.state_dict(),
              "q1_optimizer_state_dict": self.q1_optimizer.state_dict(),
              "q2_optimizer_state_dict": self.q2_optimizer.state_dict(),
              "alpha": self.alpha}
        if self.automatic_entropy_tuning:
            ck["log_alpha"] = self.log_alpha.detach().clone().requires_grad_(True)
            ck["alpha_optimizer_state_dict"] = self.alpha_optimizer.state_dict()
        if replay_buffer:
            # the reference pickles its deque of tuples; stored here as plain arrays so
            # the checkpoint loads with torch.load(weights_only=True)
            # (an empty replay is saved too: loading it empties the buffer, as assigning
            # the reference's empty deque does)
            n = len(self.replay_buffer)
            S, A = self._cfg.state_dim, self._cfg.action_dim
            if n:
                s, a, r, s2, d = self.replay_buffer._rows_at(np.arange(n))
            else:
                s, a, r, s2 = (np.zeros((0, S), np.float32), np.zeros((0, A), np.float32),
                               np.zeros(0, np.float32), np.zeros((0, S), np.float32))
                d = np.zeros(0, bool)
            ck["replay_buffer"] = {"state": torch.from_numpy(s), "action": torch.from_numpy(a),
                                   "reward": torch.from_numpy(r),
                                   "next_state": torch.from_numpy(s2),
                                   "done": torch.from_numpy(d)}
        # NB: the reference only calls torch.save when replay_buffer=True (an
        # indentation slip at sac_imp.py:198-201); the drop-in always saves.
        torch.save(ck, path)

    def load_checkpoint(self, path, load_replay_buffer=True):
        ck = _load_checkpoint_file(path)
        # the replay rows are checked before anything is overwritten (a checkpoint whose rows
        # do not fit this agent leaves it untouched), and replace the buffer at the end, as
        # the reference's assignment does (sac_imp.py:229-230)
        rows = None
        if load_replay_buffer and "replay_buffer" in ck:
            rows = self._checkpoint_rows(ck["replay_buffer"])
        self._load_nets(ck)
        for name in ("policy", "q1", "q2"):
            key = f"{name}_optimizer_state_dict"
            if key in ck:
                getattr(self, f"{name}_optimizer").load_state_dict(ck[key])
        self.alpha = ck["alpha"]
        if self.automatic_entropy_tuning and "log_alpha" in ck:
            self.log_alpha = ck["log_alpha"]
        if "alpha_optimizer_state_dict" in ck and self.automatic_entropy_tuning:
            self.alpha_optimizer.load_state_dict(ck["alpha_optimizer_state_dict"])
        if rows is not None:
            self.replay_buffer._replace_arrays(*rows)
        return ck.get("episode", 0), ck.get("total_steps", 0)

    def _checkpoint_rows(self, rb):
        """The checkpoint's replay as stacked float32 arrays (s, a, r, s2, d), shape-checked
        against this agent: the drop-in's dict of tensors, or the reference's sequence of
        (state, action, reward, next_state, done) tuples."""
        S, A = self._cfg.state_dim, self._cfg.action_dim
        if isinstance(rb, dict):
            s, a, r, s2, d = (np.asarray(rb[k].numpy() if torch.is_tensor(rb[k]) else rb[k])
                              for k in ("state", "action", "reward", "next_state", "done"))
        else:
            rb = list(rb)
            if not rb:
                z = np.zeros((0, S), np.float32)
                return z, np.zeros((0, A), np.float32), np.zeros(0, np.float32), z, np.zeros(0, bool)
            s, a, r, s2, d = (np.asarray(x) for x in zip(*rb))
        n = len(r)
        try:
            out = (np.asarray(s, np.float32).reshape(n, S), np.asarray(a, np.float32).reshape(n, A),
                   np.asarray(r, np.float32).reshape(n), np.asarray(s2, np.float32).reshape(n, S),
                   np.asarray(d).astype(bool).reshape(n))
        except ValueError as e:
            raise ValueError(f"checkpoint replay rows do not fit state_dim={S}, action_dim={A}: {e}")
        return out
