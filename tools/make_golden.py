#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ by RUNNING THE REFERENCE.

Runs only in the build container (needs /root/reference; the GPU box never does).
The reference is imported from /root/reference (read-only), driven through its own
public API (``SAC(...)``, ``agent.replay_buffer.push``, ``agent.update_parameters``,
``PrioritizedReplayBuffer``), and its inputs/outputs are written as plain arrays.
No reference source is copied.

Fixtures
--------
step_small.npz     S=24 A=4 H=64 B=32, 300 rows, two consecutive updates: every
                   input (params, rows, MT state, the two eps draws) and every output
                   (losses, all params, Adam m/v/step, log_alpha, alpha).
step_model2.npz    as step_small with networks_model2 (3 hidden layers) swapped into the
                   reference SAC.
init_seed3.npz     the reference's own init under torch.manual_seed(3) (model1; model2).
step_humanoid.npz  S=376 A=17 H=512 B=256, 2000 rows (state scale 0.1), two updates:
                   inputs regenerable from PCG64 seeds; outputs = losses, per-tensor
                   norms of the parameter deltas and strided element samples.
idx_uniform.npz    random.sample(deque, k) index vectors for both sample branches.
per.npz            PrioritizedReplayBuffer.sample / update_priorities vectors.

Usage:  python tools/make_golden.py [--out tests/golden]
"""
from __future__ import annotations

import argparse
import os
import random
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
sys.path.insert(0, REPO)
from oracle.pyrandom import MT19937, sample_indices            # noqa: E402
from oracle.sac_step import (SacConfig, init_params, synthetic_rows,  # noqa: E402
                             NETS, OracleSAC)

STRIDE = 61   # strided element sample for the big fixture


def _ref_modules():
    sys.path.insert(0, REF)
    import sac_imp            # noqa: F401  (reference)
    import replay_buffer      # noqa: F401  (reference)
    return sys.modules["sac_imp"], sys.modules["replay_buffer"]


class _model2_swap:
    """The reference's SAC with networks_model2 in place of networks_model1 — the swap its
    author makes by editing sac_imp.py:4 (the import line).  networks_model2's policy
    defaults to device="cuda" (networks_model2.py:52); the build container has none, so
    the class is wrapped to pass device="cpu" (nothing else changes)."""

    def __enter__(self):
        sac_imp, _ = _ref_modules()
        import networks_model2 as m2   # noqa: F401  (reference)
        self.saved = (sac_imp.QNetwork, sac_imp.GaussianPolicy)

        class _Policy(m2.GaussianPolicy):
            def __init__(self, s, a, h=512, device="cpu", action_bounds=None):
                super().__init__(s, a, h, device="cpu", action_bounds=action_bounds)

        sac_imp.QNetwork, sac_imp.GaussianPolicy = m2.QNetwork, _Policy
        return self

    def __exit__(self, *exc):
        sac_imp, _ = _ref_modules()
        sac_imp.QNetwork, sac_imp.GaussianPolicy = self.saved


def _load_into_ref(agent, params):
    for n in NETS:
        sd = {k: torch.from_numpy(v.copy()) for k, v in params[n].items()}
        getattr(agent, n).load_state_dict(sd)


def _ref_state(agent) -> dict:
    out = {}
    for n in NETS:
        for k, v in getattr(agent, n).state_dict().items():
            out[f"{n}.{k}"] = v.detach().numpy().copy()
    for n, opt in (("policy", agent.policy_optimizer), ("q1", agent.q1_optimizer),
                   ("q2", agent.q2_optimizer)):
        net = getattr(agent, n)
        for (k, p) in net.named_parameters():
            st = opt.state.get(p, {})
            if st:
                out[f"adam.{n}.{k}.m"] = st["exp_avg"].numpy().copy()
                out[f"adam.{n}.{k}.v"] = st["exp_avg_sq"].numpy().copy()
                out[f"adam.{n}.step"] = np.array(float(st["step"]))
    out["log_alpha"] = agent.log_alpha.detach().numpy().copy()
    st = agent.alpha_optimizer.state.get(agent.log_alpha, {})
    if st:
        out["adam.log_alpha.m"] = st["exp_avg"].numpy().copy()
        out["adam.log_alpha.v"] = st["exp_avg_sq"].numpy().copy()
    a = agent.alpha
    out["alpha"] = np.array(float(a) if not torch.is_tensor(a) else float(a.detach()))
    return out


def run_reference(cfg: SacConfig, params, rows, batch, steps, py_seed, torch_seed):
    """Drive the reference SAC for ``steps`` updates; capture inputs and outputs."""
    sac_imp, _ = _ref_modules()
    agent = sac_imp.SAC(cfg.state_dim, cfg.action_dim, hidden_dim=cfg.hidden_dim,
                        gamma=cfg.gamma, tau=cfg.tau, lr=cfg.lr, alpha=cfg.alpha,
                        automatic_entropy_tuning=cfg.automatic_entropy_tuning, device="cpu")
    _load_into_ref(agent, params)
    s, a, r, s2, d = rows
    for i in range(len(r)):   # the trainer pushes float64 states, float32 actions
        agent.replay_buffer.push(s[i].astype(np.float64), a[i].copy(), float(r[i]),
                                 s2[i].astype(np.float64), bool(d[i]))
    random.seed(py_seed)
    torch.manual_seed(torch_seed)
    rec = []
    for _ in range(steps):
        pre_py = random.getstate()
        pre_torch = torch.get_rng_state()
        losses = agent.update_parameters(batch)
        post_py = random.getstate()
        post_torch = torch.get_rng_state()
        # recover the draws the update consumed (nothing else touches the streams)
        mt = MT19937.from_pystate(pre_py)
        idx = sample_indices(mt, len(agent.replay_buffer), batch)
        assert mt.to_pystate() == post_py
        torch.set_rng_state(pre_torch)
        e1 = torch.empty(batch, cfg.action_dim).normal_()
        e2 = torch.empty(batch, cfg.action_dim).normal_()
        assert torch.equal(torch.get_rng_state(), post_torch)
        rec.append(dict(mt_key=MT19937.from_pystate(pre_py).key, mt_pos=pre_py[1][624],
                        idx=idx, eps1=e1.numpy().copy(), eps2=e2.numpy().copy(),
                        losses=np.array([losses["q1_loss"], losses["q2_loss"],
                                         losses["policy_loss"]], dtype=np.float64),
                        state=_ref_state(agent)))
    return rec


def check_oracle_bitexact(cfg, params, rows, rec):
    """The fp32 oracle must reproduce the reference bit for bit."""
    orc = OracleSAC(cfg, params, dtype=torch.float32)
    s, a, r, s2, d = rows
    worst = 0.0
    for st in rec:
        i = st["idx"]
        L = orc.step(s[i], a[i], r[i], s2[i], d[i], st["eps1"], st["eps2"])
        assert np.array_equal(np.array([L["q1_loss"], L["q2_loss"], L["policy_loss"]]),
                              st["losses"]), (L, st["losses"])
        mine = orc.state()
        for k, v in st["state"].items():
            diff = float(np.max(np.abs(np.asarray(mine[k], np.float64) - np.asarray(v, np.float64))))
            worst = max(worst, diff)
            assert np.array_equal(np.asarray(mine[k]), np.asarray(v)), k
    return worst


def make_step_small(out):
    cfg = SacConfig(24, 4, 64)
    params = init_params(cfg, seed=11, bias_scale=0.05)
    rows = synthetic_rows(cfg, 300, seed=12, state_scale=0.5)
    rec = run_reference(cfg, params, rows, batch=32, steps=2, py_seed=13, torch_seed=14)
    check_oracle_bitexact(cfg, params, rows, rec)
    blob = {"cfg": np.array([24, 4, 64, 32, 300])}
    for n in NETS:
        for k, v in params[n].items():
            blob[f"in.{n}.{k}"] = v
    for name, arr in zip(("s", "a", "r", "s2", "d"), rows):
        blob[f"rows.{name}"] = arr
    for t, st in enumerate(rec):
        for k in ("mt_key", "mt_pos", "idx", "eps1", "eps2", "losses"):
            blob[f"step{t}.{k}"] = np.asarray(st[k])
        for k, v in st["state"].items():
            blob[f"step{t}.out.{k}"] = np.asarray(v)
    np.savez_compressed(os.path.join(out, "step_small.npz"), **blob)
    print("step_small.npz: oracle fp32 == reference bit-exact over 2 updates")


def make_step_model2(out):
    """networks_model2 (3 hidden layers, orthogonal policy init) in the reference SAC."""
    cfg = SacConfig(24, 4, 64, n_hidden=3)
    params = init_params(cfg, seed=31, bias_scale=0.05)
    rows = synthetic_rows(cfg, 300, seed=32, state_scale=0.5)
    with _model2_swap():
        rec = run_reference(cfg, params, rows, batch=32, steps=2, py_seed=33, torch_seed=34)
    check_oracle_bitexact(cfg, params, rows, rec)
    blob = {"cfg": np.array([24, 4, 64, 32, 300, 3])}
    for n in NETS:
        for k, v in params[n].items():
            blob[f"in.{n}.{k}"] = v
    for name, arr in zip(("s", "a", "r", "s2", "d"), rows):
        blob[f"rows.{name}"] = arr
    for t, st in enumerate(rec):
        for k in ("mt_key", "mt_pos", "idx", "eps1", "eps2", "losses"):
            blob[f"step{t}.{k}"] = np.asarray(st[k])
        for k, v in st["state"].items():
            blob[f"step{t}.out.{k}"] = np.asarray(v)
    np.savez_compressed(os.path.join(out, "step_model2.npz"), **blob)
    print("step_model2.npz: oracle fp32 == reference (networks_model2) bit-exact over 2 updates")


def make_step_humanoid(out):
    cfg = SacConfig(376, 17, 512)
    P_SEED, R_SEED = 21, 22
    params = init_params(cfg, seed=P_SEED, bias_scale=0.02)
    rows = synthetic_rows(cfg, 2000, seed=R_SEED, state_scale=0.1)
    rec = run_reference(cfg, params, rows, batch=256, steps=2, py_seed=23, torch_seed=24)
    check_oracle_bitexact(cfg, params, rows, rec)
    blob = {"cfg": np.array([376, 17, 512, 256, 2000]),
            "seeds": np.array([P_SEED, R_SEED]), "bias_scale": np.array(0.02),
            "state_scale": np.array(0.1), "stride": np.array(STRIDE)}
    prev = {f"{n}.{k}": v for n in NETS for k, v in params[n].items()}
    for t, st in enumerate(rec):
        for k in ("mt_key", "mt_pos", "idx", "eps1", "eps2", "losses"):
            blob[f"step{t}.{k}"] = np.asarray(st[k])
        for k, v in st["state"].items():
            v = np.asarray(v)
            if k in prev:
                blob[f"step{t}.dnorm.{k}"] = np.array(np.linalg.norm((v - prev[k]).astype(np.float64)))
            blob[f"step{t}.sample.{k}"] = v.reshape(-1)[::STRIDE].copy()
        prev = {k: np.asarray(v) for k, v in st["state"].items() if k in prev}
    np.savez_compressed(os.path.join(out, "step_humanoid.npz"), **blob)
    print("step_humanoid.npz: oracle fp32 == reference bit-exact over 2 updates")


def make_idx(out):
    _, replay_buffer = _ref_modules()
    cases = [(0, 300, 256), (1, 1045, 256), (2, 1046, 256), (3, 20000, 256),
             (4, 1000000, 256), (5, 257, 256), (6, 16405, 4096), (7, 16406, 4096),
             (8, 200000, 4096), (9, 64, 1), (10, 6, 6), (11, 100, 5)]
    blob = {"cases": np.array(cases, dtype=np.int64)}
    for c, (seed, n, k) in enumerate(cases):
        buf = replay_buffer.ReplayBuffer(capacity=max(n, 1))
        for i in range(n):   # rows carry their own position as the state
            buf.push(np.array([float(i)]), np.zeros(1, np.float32), 0.0, np.zeros(1), False)
        random.seed(seed)
        pre = random.getstate()
        st, *_ = buf.sample(k)
        post = random.getstate()
        blob[f"c{c}.key"] = np.array(pre[1][:624], dtype=np.uint32)
        blob[f"c{c}.pos"] = np.array(pre[1][624])
        blob[f"c{c}.idx"] = st[:, 0].astype(np.int64)
        blob[f"c{c}.post_key"] = np.array(post[1][:624], dtype=np.uint32)
        blob[f"c{c}.post_pos"] = np.array(post[1][624])
    np.savez_compressed(os.path.join(out, "idx_uniform.npz"), **blob)
    print("idx_uniform.npz:", len(cases), "cases")


def make_per(out):
    _, replay_buffer = _ref_modules()
    blob = {}
    cases = [(0, 50, 16, 64), (1, 1000, 256, 1000), (2, 5000, 256, 4096), (3, 3000, 4096, 3000)]
    blob["cases"] = np.array(cases, dtype=np.int64)
    for c, (seed, n, batch, cap) in enumerate(cases):
        rng = np.random.default_rng(100 + seed)
        buf = replay_buffer.PrioritizedReplayBuffer(cap)
        pushed_prios = []
        for i in range(n):
            buf.push(np.array([float(i)], np.float32), np.zeros(1, np.float32), 0.0,
                     np.zeros(1, np.float32), False)
            if i % 97 == 5:     # occasionally raise priorities mid-stream
                ids = rng.integers(0, min(i + 1, cap), size=3)
                pr = rng.uniform(0.01, 3.0, size=3).astype(np.float32)
                buf.update_priorities(ids, torch.from_numpy(pr))
                pushed_prios.append((i, ids, pr))
        blob[f"c{c}.prio_before"] = buf.priorities.copy()
        np.random.seed(200 + seed)
        st = np.random.get_state()
        blob[f"c{c}.np_key"] = st[1].astype(np.uint32)
        blob[f"c{c}.np_pos"] = np.array(st[2])
        blob[f"c{c}.frame"] = np.array(buf.frame)
        probs = buf.priorities[:len(buf.buffer)] ** buf.alpha
        probs /= probs.sum()
        blob[f"c{c}.probs"] = probs
        states, _, _, _, _, idx, w = buf.sample(batch)
        post = np.random.get_state()
        blob[f"c{c}.idx"] = np.asarray(idx, np.int64)
        blob[f"c{c}.weights"] = np.asarray(w, np.float32)
        blob[f"c{c}.states"] = states[:, 0].copy()
        blob[f"c{c}.np_post_pos"] = np.array(post[2])
        blob[f"c{c}.np_post_key"] = post[1].astype(np.uint32)
        newp = rng.uniform(0.0, 5.0, size=len(idx)).astype(np.float32)
        buf.update_priorities(idx, torch.from_numpy(newp))
        blob[f"c{c}.upd_prio"] = newp
        blob[f"c{c}.prio_after"] = buf.priorities.copy()
        # one more push after the update: max priority over the whole array
        buf.push(np.array([-1.0], np.float32), np.zeros(1, np.float32), 0.0,
                 np.zeros(1, np.float32), False)
        blob[f"c{c}.prio_after_push"] = buf.priorities.copy()
        blob[f"c{c}.pos_after_push"] = np.array(buf.pos)
    np.savez_compressed(os.path.join(out, "per.npz"), **blob)
    print("per.npz:", len(cases), "cases")


def make_init(out):
    """The reference's own initialisation (nn.Linear + xavier_uniform_/zero bias in
    SAC.__init__ construction order) under torch.manual_seed(3)."""
    sac_imp, _ = _ref_modules()
    blob = {}
    for (S, A, H) in ((24, 4, 64), (376, 17, 256)):
        torch.manual_seed(3)
        agent = sac_imp.SAC(S, A, hidden_dim=H, device="cpu")
        for n in NETS:
            for k, v in getattr(agent, n).state_dict().items():
                blob[f"{S}_{A}_{H}.{n}.{k}"] = v.numpy().copy()
    with _model2_swap():     # networks_model2: orthogonal policy init (networks_model2.py:82)
        S, A, H = 24, 4, 64
        torch.manual_seed(3)
        agent = sac_imp.SAC(S, A, hidden_dim=H, device="cpu")
        for n in NETS:
            for k, v in getattr(agent, n).state_dict().items():
                blob[f"m2_{S}_{A}_{H}.{n}.{k}"] = v.numpy().copy()
    np.savez_compressed(os.path.join(out, "init_seed3.npz"), **blob)
    print("init_seed3.npz")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(REPO, "tests", "golden"))
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    torch.set_num_threads(8)
    todo = args.only.split(",") if args.only else ["idx", "per", "small", "humanoid", "init", "model2"]
    if "init" in todo:
        make_init(args.out)
    if "idx" in todo:
        make_idx(args.out)
    if "per" in todo:
        make_per(args.out)
    if "small" in todo:
        make_step_small(args.out)
    if "humanoid" in todo:
        make_step_humanoid(args.out)
    if "model2" in todo:
        make_step_model2(args.out)


if __name__ == "__main__":
    main()
