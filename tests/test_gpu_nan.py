"""Non-finite inputs raise ValueError where the reference raises, and leave the state the
reference leaves (include/sacmi.h SACMI_ENAN, csrc/sacmi_internal.h ErrBits):

* Normal(mean, std) validates its arguments (networks_model1.py:87, torch
  distributions `_validate_args`): a NaN policy mean / log_std in
  policy.sample(next_state) raises before any step (sac_imp.py:89), in
  policy.sample(state) after the critic step and before the actor / alpha / Polyak steps
  (sac_imp.py:116); select_action(evaluate=False) raises, evaluate=True does not.
* np.random.choice(p=probs) raises "probabilities contain NaN" (replay_buffer.py:60-64):
  the frame has advanced (:54-55), the numpy stream has not.
"""
import random

import numpy as np
import pytest
import torch

from oracle.pyrandom import MT19937, sample_indices

pytestmark = pytest.mark.gpu

S, A, H = 24, 4, 64
NETS = ("policy", "q1", "q2", "q1_target", "q2_target")


def _agent(**kw):
    from sac_imp import SAC
    torch.manual_seed(0)
    return SAC(S, A, hidden_dim=H, device="cuda", capacity=5000, max_batch=256, seed=11, **kw)


def _fill(agent, n, seed=0, nan_state_rows=()):
    rng = np.random.default_rng(seed)
    for i in range(n):
        s = rng.standard_normal(S)
        if i in nan_state_rows:
            s[3] = np.nan
        agent.replay_buffer.push(s, rng.uniform(-0.4, 0.4, A).astype(np.float32),
                                 float(rng.standard_normal()), rng.standard_normal(S),
                                 bool(rng.random() < 0.02))


def _snapshot(ctx):
    from sacmi import _lib as L
    snap = {f"{n}.{k}": v for n in NETS for k, v in ctx.get_net(n).items()}
    for n in ("policy", "q1", "q2"):
        for slot in ("m", "v"):
            snap.update({f"{n}.{slot}.{k}": v for k, v in ctx.get_net(n, slot).items()})
    for sid in (L.S_STEP_POLICY, L.S_STEP_Q1, L.S_STEP_Q2, L.S_STEP_ALPHA, L.S_LOG_ALPHA,
                L.S_ALPHA, L.S_ADAM_M_LOG_ALPHA, L.S_ADAM_V_LOG_ALPHA):
        snap[f"scalar{sid}"] = np.array(ctx.get_scalar(sid))
    return snap


def _same(a, b, keys):
    for k in keys:
        assert np.array_equal(a[k], b[k], equal_nan=True), k


def _poison_policy(ctx, value=np.nan):
    w = ctx.get_tensor("param", "policy", 1, 0, (H, H))     # policy.fc2.weight
    w[3, 5] = value
    ctx.set_tensor("param", "policy", 1, 0, w)
    return w


def test_nan_policy_update_raises_and_takes_no_step():
    """A NaN in policy.fc2.weight: every policy output is NaN, so update_parameters raises
    at policy.sample(next_state) (sac_imp.py:89) — no parameter, moment, step count, alpha
    or target changes; the update's random.sample has consumed the stream, as the
    reference's had (sac_imp.py:77-78 runs first).  Fixing the weight, the next update runs."""
    agent = _agent(sync_python_random=True)
    _fill(agent, 300)
    agent.update_parameters(64)
    agent.update_parameters(64)
    w = _poison_policy(agent._ctx)
    before = _snapshot(agent._ctx)
    random.seed(5)
    pre = random.getstate()
    with pytest.raises(ValueError, match=r"Normal.*next_state_batch"):
        agent.update_parameters(64)
    after = _snapshot(agent._ctx)
    _same(before, after, before.keys())
    mt = MT19937.from_pystate(pre)
    sample_indices(mt, 300, 64)
    assert random.getstate() == mt.to_pystate()
    # the flag is gone once reported: fix the weight and train on
    w[3, 5] = 0.01
    agent._ctx.set_tensor("param", "policy", 1, 0, w)
    out = agent.update_parameters(64)
    assert all(np.isfinite(v) for v in out.values())
    from sacmi import _lib as L
    assert agent._ctx.get_scalar(L.S_STEP_POLICY) == before[f"scalar{L.S_STEP_POLICY}"] + 1


def test_nan_policy_many_updates_stop_at_the_first():
    """update_parameters_many(n) is the trainer's loop (trainer.py:203-204): it raises at
    its first update and the later updates of the launch take no step and draw nothing —
    the state equals that of one failed update_parameters."""
    a1, a2 = _agent(), _agent()
    for ag in (a1, a2):
        _fill(ag, 300)
        ag.update_parameters(64)
        _poison_policy(ag._ctx)
    with pytest.raises(ValueError, match="Normal"):
        a1.update_parameters(64)
    with pytest.raises(ValueError, match="Normal"):
        a2.update_parameters_many(64, 5)
    s1, s2 = _snapshot(a1._ctx), _snapshot(a2._ctx)
    _same(s1, s2, s1.keys())
    assert a1._ctx.get_mt(0)[1] == a2._ctx.get_mt(0)[1]
    assert np.array_equal(a1._ctx.get_mt(0)[0], a2._ctx.get_mt(0)[0])


def test_nan_actor_batch_takes_the_critic_step_only():
    """A NaN state in the replay: policy.sample(next_state) is finite, so the critic step
    runs (on a NaN loss, as the reference's does), then policy.sample(state) raises
    (sac_imp.py:116): q1 / q2 step counts advance, the policy / alpha counts, the policy,
    log_alpha and the targets (Polyak comes last, sac_imp.py:138) do not."""
    from sacmi import _lib as L
    agent = _agent()
    _fill(agent, 64, nan_state_rows=(17,))
    before = _snapshot(agent._ctx)
    with pytest.raises(ValueError, match=r"Normal.*\bstate_batch"):
        agent.update_parameters(64)        # all 64 rows: the NaN row is in the batch
    after = _snapshot(agent._ctx)
    for sid in (L.S_STEP_Q1, L.S_STEP_Q2):
        assert after[f"scalar{sid}"] == before[f"scalar{sid}"] + 1
    keep = [k for k in before if k.startswith(("policy.", "q1_target.", "q2_target."))]
    keep += [f"scalar{sid}" for sid in (L.S_STEP_POLICY, L.S_STEP_ALPHA, L.S_LOG_ALPHA, L.S_ALPHA,
                                        L.S_ADAM_M_LOG_ALPHA, L.S_ADAM_V_LOG_ALPHA)]
    _same(before, after, keep)
    assert not np.array_equal(before["q1.fc1.weight"], after["q1.fc1.weight"], equal_nan=True)


def test_select_action_nan_raises_only_when_sampling():
    agent = _agent()
    _poison_policy(agent._ctx)
    st = np.random.default_rng(2).standard_normal(S).astype(np.float32)
    with pytest.raises(ValueError, match="select_action"):
        agent.select_action(st)
    with pytest.raises(ValueError, match="select_action"):
        agent.select_action(np.zeros((100, S)))     # the batched (copy) path too
    a = agent.select_action(st, evaluate=True)      # tanh(mean): no Normal is built
    assert np.all(np.isnan(a))
    w = agent._ctx.get_tensor("param", "policy", 1, 0, (H, H))
    w[3, 5] = 0.0
    agent._ctx.set_tensor("param", "policy", 1, 0, w)
    assert np.all(np.isfinite(agent.select_action(st)))


@pytest.mark.parametrize("bad", [np.nan, np.inf, -1.0, "zeros"])
def test_per_sample_nan_probabilities(bad):
    """PrioritizedReplayBuffer.sample with a NaN (or inf, negative: NaN after **alpha / the
    normalisation; all zero: 0/0) priority raises "probabilities contain NaN"
    (replay_buffer.py:60-64); the frame has advanced, the numpy stream has not — restored,
    the next draw equals that of a buffer that never saw the bad priority."""
    from sacmi import Config, Context
    from sacmi import _lib as L
    ctxs = [Context(Config(S, A, H, max_batch=256, capacity=20000, replay="per"), 0) for _ in range(2)]
    rng = np.random.default_rng(3)
    rows = (rng.standard_normal((20000, S)).astype(np.float32),
            rng.uniform(-0.4, 0.4, (20000, A)).astype(np.float32),
            rng.standard_normal(20000).astype(np.float32),
            rng.standard_normal((20000, S)).astype(np.float32), rng.random(20000) < 0.02)
    prio = rng.uniform(0.1, 2.0, 20000).astype(np.float32)
    for c in ctxs:
        c.push(*rows)
        c.per_set_priorities(prio)
    p2 = np.zeros_like(prio) if bad == "zeros" else prio.copy()
    if bad != "zeros":
        p2[12345] = bad
    ctxs[0].per_set_priorities(p2)
    key0, pos0 = ctxs[0].get_mt(1)
    f0 = ctxs[0].get_scalar(L.S_PER_FRAME)
    with pytest.raises(ValueError, match="probabilities contain NaN"):
        ctxs[0].per_sample(256)
    key1, pos1 = ctxs[0].get_mt(1)
    assert pos1 == pos0 and np.array_equal(key1, key0)
    assert ctxs[0].get_scalar(L.S_PER_FRAME) == f0 + 1
    ctxs[0].per_set_priorities(prio)
    ctxs[1].set_scalar(L.S_PER_FRAME, f0 + 1)
    i0, w0 = ctxs[0].per_sample(256)
    i1, w1 = ctxs[1].per_sample(256)
    assert np.array_equal(i0, i1) and np.array_equal(w0, w1)
    for c in ctxs:
        c.close()


def test_per_update_nan_probabilities_take_no_step():
    """A prioritized-replay update (device sampling inside the update graph) with a NaN
    priority: the update raises before any step; frame +1, numpy stream untouched."""
    from sacmi import Config, Context
    from sacmi import _lib as L
    ctx = Context(Config(S, A, H, max_batch=256, capacity=4096, replay="per"), 0)
    rng = np.random.default_rng(4)
    ctx.push(rng.standard_normal((4096, S)).astype(np.float32),
             rng.uniform(-0.4, 0.4, (4096, A)).astype(np.float32),
             rng.standard_normal(4096).astype(np.float32),
             rng.standard_normal((4096, S)).astype(np.float32), rng.random(4096) < 0.02)
    ctx.step(64)
    p = ctx.per_priorities(4096)
    p[7] = np.nan
    ctx.per_set_priorities(p)
    before = _snapshot(ctx)
    key0, pos0 = ctx.get_mt(1)
    f0 = ctx.get_scalar(L.S_PER_FRAME)
    with pytest.raises(ValueError, match="probabilities contain NaN"):
        ctx.step(64)
    _same(before, _snapshot(ctx), before.keys())
    key1, pos1 = ctx.get_mt(1)
    assert pos1 == pos0 and np.array_equal(key1, key0)
    assert ctx.get_scalar(L.S_PER_FRAME) == f0 + 1
    ctx.close()


def test_nan_split_k_bf16_and_phase_paths():
    """The other Adam epilogues: the bf16 split-K weight-gradient levels (k_dw_fin, batch
    2048, with the next update's sampling riding in L6) in a multi-update launch, and the
    data-parallel phase split (k_adam) — both stop at the NaN sample without a step."""
    from sacmi import Config, Context
    for mode in ("bf16_many", "phases"):
        bf = mode == "bf16_many"
        B = 2048 if bf else 64
        ctx = Context(Config(S, A, 256 if bf else H, max_batch=B, capacity=8192,
                             compute_dtype="bf16" if bf else "fp32"), 0)
        rng = np.random.default_rng(6)
        ctx.push(rng.standard_normal((8192, S)).astype(np.float32),
                 rng.uniform(-0.4, 0.4, (8192, A)).astype(np.float32),
                 rng.standard_normal(8192).astype(np.float32),
                 rng.standard_normal((8192, S)).astype(np.float32), rng.random(8192) < 0.02)
        hh = 256 if bf else H
        w = ctx.get_tensor("param", "policy", 1, 0, (hh, hh))
        w[3, 5] = np.nan
        ctx.set_tensor("param", "policy", 1, 0, w)
        before = _snapshot(ctx)
        key0, pos0 = ctx.get_mt(0)
        if bf:
            ctx.step_many_async(B, 4)
        else:
            for ph in (0, 1, 2):
                ctx.step_phase(B, ph)
        with pytest.raises(ValueError, match="Normal"):
            ctx.fetch_losses(8)
        _same(before, _snapshot(ctx), before.keys())
        key1, pos1 = ctx.get_mt(0)
        mt = MT19937(np.asarray(key0, np.uint32), pos0)
        sample_indices(mt, 8192, B)              # the first update's draw only
        assert pos1 == mt.pos and np.array_equal(key1, np.asarray(mt.key, np.uint32)), mode
        ctx.close()


@pytest.mark.parametrize("sharded", [False, True])
def test_dp_remote_nan_voids_the_update_on_every_rank(sharded):
    """Data parallel: a rank whose update sees a non-finite input (another rank, emulated by
    the loopback's SACMI_DP_LOOPBACK_REMOTE_ERR) makes every rank void the same steps — the
    error flags travel with the critic gradient collective (csrc/sacmi_internal.h kDpFlagN),
    so no rank applies a partial update and the replicas stay identical.  This rank's own
    inputs are finite: its update raises ValueError naming the other rank, takes no step, and
    the launch's later updates draw nothing (the first update's random.sample only)."""
    import os
    from sacmi import Config, Context
    B = 64
    ctx = Context(Config(S, A, H, max_batch=B, capacity=4096), 0)
    rng = np.random.default_rng(8)
    ctx.push(rng.standard_normal((4096, S)).astype(np.float32),
             rng.uniform(-0.4, 0.4, (4096, A)).astype(np.float32),
             rng.standard_normal(4096).astype(np.float32),
             rng.standard_normal((4096, S)).astype(np.float32), rng.random(4096) < 0.02)
    ctx.dp_loopback_init(2)
    ctx.dp_set_sharded(sharded)
    before = _snapshot(ctx)
    key0, pos0 = ctx.get_mt(0)
    os.environ["SACMI_DP_LOOPBACK_REMOTE_ERR"] = "1"
    try:
        ctx.step_dp(B, 3)
        ctx.synchronize()
    finally:
        os.environ.pop("SACMI_DP_LOOPBACK_REMOTE_ERR", None)
    with pytest.raises(ValueError, match="another data-parallel rank"):
        ctx.fetch_losses(8)
    _same(before, _snapshot(ctx), before.keys())
    key1, pos1 = ctx.get_mt(0)
    mt = MT19937(np.asarray(key0, np.uint32), pos0)
    sample_indices(mt, 4096, B)
    assert pos1 == mt.pos and np.array_equal(key1, np.asarray(mt.key, np.uint32))
    ctx.close()
