"""Oracle backend for sacmi.dp.DataParallelUpdate (test infrastructure).

Splits the oracle's SAC update into the library's three phases with explicit flat
gradient buffers, so the SAME DataParallelUpdate driver that runs the GPU path can be
exercised with the gloo backend on CPU.
"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "humanoid-walking-with-sac_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

from oracle.sac_step import (NETS, Q_KEYS, OracleSAC, _policy_sample,  # noqa: E402
                             _q_forward)


class OraclePhases(OracleSAC):
    """OracleSAC whose update is driven phase by phase (test-only)."""

    def __post_init__(self):
        super().__post_init__()
        nq = sum(v.numel() for n in ("q1", "q2") for v in self.nets[n].values())
        npi = sum(v.numel() for v in self.nets["policy"].values())
        self.critic_grads = torch.zeros(nq, dtype=self.dtype)
        self.actor_grads = torch.zeros(npi + 1, dtype=self.dtype)
        self.batch = None

    def set_batch(self, s, a, r, s2, d, eps1, eps2):
        T = lambda x: torch.as_tensor(np.asarray(x, dtype=np.float32)).to(self.dtype)
        self.batch = (T(s), T(a), T(r).reshape(-1, 1), T(s2), T(d).reshape(-1, 1), T(eps1), T(eps2))

    def _flat_into(self, buf, tensors):
        o = 0
        for t in tensors:
            n = t.numel()
            buf[o:o + n] = t.reshape(-1)
            o += n

    def _grads_from(self, buf, params, scale):
        o = 0
        for p in params:
            n = p.numel()
            p.grad = (buf[o:o + n] * scale).reshape(p.shape).clone()
            o += n

    def phase(self, p, batch, grad_scale):
        cfg = self.cfg
        state, action, reward, next_state, done, e1, e2 = self.batch
        P, Q1, Q2 = self.nets["policy"], self.nets["q1"], self.nets["q2"]
        sc, bi = cfg.action_scale, cfg.action_bias
        qparams = [Q1[k] for k in Q_KEYS] + [Q2[k] for k in Q_KEYS]
        pparams = list(P.values())
        if p == 0:
            with torch.no_grad():
                na, nlp = _policy_sample(P, next_state, e1, sc, bi)
                q1n = _q_forward(self.nets["q1_target"], next_state, na)
                q2n = _q_forward(self.nets["q2_target"], next_state, na)
                q_target = reward + (1 - done) * cfg.gamma * (torch.min(q1n, q2n) - self.alpha * nlp)
            l1 = F.mse_loss(_q_forward(Q1, state, action), q_target)
            l2 = F.mse_loss(_q_forward(Q2, state, action), q_target)
            g = torch.autograd.grad(l1 + l2, qparams)   # disjoint params: sum == each
            self._flat_into(self.critic_grads, g)
        elif p == 1:
            self._grads_from(self.critic_grads, qparams, grad_scale)
            self.opt["q1"].step()
            self.opt["q2"].step()
            for q in qparams:
                q.grad = None
            with torch.no_grad():   # Polyak (targets are not read again this update)
                for src, dst in (("q1", "q1_target"), ("q2", "q2_target")):
                    for k in Q_KEYS:
                        t = self.nets[dst][k]
                        t.copy_(t * (1.0 - cfg.tau) + self.nets[src][k] * cfg.tau)
            new_a, logp = _policy_sample(P, state, e2, sc, bi)
            q_new = torch.min(_q_forward(Q1, state, new_a), _q_forward(Q2, state, new_a))
            alpha = self.alpha.detach() if torch.is_tensor(self.alpha) else self.alpha
            policy_loss = (alpha * logp - q_new).mean()
            g = torch.autograd.grad(policy_loss, pparams)
            self._flat_into(self.actor_grads[:-1], g)
            self.actor_grads[-1] = -(logp.detach() + (-cfg.action_dim)).mean()
        elif p == 2:
            self._grads_from(self.actor_grads[:-1], pparams, grad_scale)
            self.opt["policy"].step()
            for q in pparams:
                q.grad = None
            if cfg.automatic_entropy_tuning:
                self.log_alpha.grad = (self.actor_grads[-1:] * grad_scale).clone()
                self.opt["alpha"].step()
                self.alpha = self.log_alpha.detach().exp()


def worker(rank, world, port, cfg, params, shards, idx, eps1, eps2, out_dir, steps):
    import torch.distributed as dist
    from sacmi.dp import DataParallelUpdate
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    be = OraclePhases(cfg, params, dtype=torch.float64)
    upd = DataParallelUpdate(be)
    rows = shards[rank]
    for t in range(steps):
        i = idx[t][rank]
        be.set_batch(*[x[i] for x in rows], eps1[t][rank], eps2[t][rank])
        upd(len(i))
    upd.flush()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **be.state())
    dist.barrier()
    dist.destroy_process_group()


def per_shard_indices(prio, n, batch, key, steps, frame0=1):
    """Per-rank prioritized sampling of a shard (replay_buffer.py:48-82 restated by
    oracle/per.py): probabilities normalised over THIS shard only, uniforms from the rank's
    own numpy MT stream, beta annealed by the rank's own frame counter."""
    from oracle.per import beta_at, probs_from, sample_from_probs
    from oracle.pyrandom import MT19937
    mt = MT19937(np.asarray(key, np.uint32), 624)
    out = []
    for t in range(steps):
        probs = probs_from(prio, n)
        idx, w = sample_from_probs(probs, batch, mt, beta_at(frame0 + t))
        out.append((idx, w))
    return out


def worker_per(rank, world, port, cfg, params, shards, prios, keys, eps1, eps2, out_dir, steps,
               batch):
    """A rank of the BASELINE configs[3] layout on CPU: its own prioritized replay shard,
    its own sampler, the production DataParallelUpdate driver over gloo."""
    import torch.distributed as dist
    from sacmi.dp import DataParallelUpdate
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    be = OraclePhases(cfg, params, dtype=torch.float64)
    upd = DataParallelUpdate(be)
    rows = shards[rank]
    draws = per_shard_indices(prios[rank], len(rows[2]), batch, keys[rank], steps)
    for t in range(steps):
        i = draws[t][0]
        be.set_batch(*[x[i] for x in rows], eps1[t][rank], eps2[t][rank])
        upd(len(i))
    upd.flush()
    st = be.state()
    for t in range(steps):
        st[f"idx{t}"] = draws[t][0]
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **st)
    dist.barrier()
    dist.destroy_process_group()
